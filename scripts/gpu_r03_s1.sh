#!/usr/bin/env bash
# Round-3 re-entry evidence in one call: the GPU suite (minus the server-overlap timing
# test, which is measured separately below), the profile round, the server-overlap
# experiment and the N = 2 rehearsal line.
#   gpurun --timeout 1200 -- bash scripts/gpu_r03_s1.sh <tag>
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="${1:-r03_s1}"
OUT="$ROOT/gpurun_out/$TAG"
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
  --deselect tests/test_gpu_hooks.py::test_batches_next_to_a_persistent_server \
  > "$OUT/pytest_gpu.log" 2>&1 || { tail -30 "$OUT/pytest_gpu.log"; exit 1; }
tail -2 "$OUT/pytest_gpu.log"
ENET_CRC_AMD_LIB="$ROOT/rusty_enet_amd/lib/variants/libenet_crc_amd_testhooks.so" timeout -k 10 170 \
  python scripts/exp_server_overlap.py > "$OUT/server_overlap.txt" 2>&1 || { tail -20 "$OUT/server_overlap.txt"; exit 1; }
cat "$OUT/server_overlap.txt"
BENCH_SHARE_GPUS=1 timeout -k 10 300 python bench.py --gpus 2 --steps 10 --warmup 2 \
  > "$OUT/bench_rehearsal_n2.json" 2> "$OUT/bench_rehearsal_n2.err" || { tail -20 "$OUT/bench_rehearsal_n2.err"; exit 1; }
bash scripts/gpu_profile_round.sh "$TAG"
