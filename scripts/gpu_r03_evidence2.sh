#!/usr/bin/env bash
# Round-3 evidence, second call: the N = 2 rehearsal line (bench.py --gpus 2 with ranks
# sharing the one GPU: large_64k + devices fields), the G1 counter diff against probe P9
# (scripts/gpu_g1_diff.sh), and the server-overlap experiment (test-hooks build).
#   gpurun --timeout 1200 -- bash scripts/gpu_r03_evidence2.sh <tag>
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="${1:-r03_ev2}"
OUT="$ROOT/gpurun_out/$TAG"
mkdir -p "$OUT"
cd "$ROOT"
BENCH_SHARE_GPUS=1 timeout -k 10 300 python bench.py --gpus 2 --steps 10 --warmup 2 \
  > "$OUT/bench_rehearsal_n2.json" 2> "$OUT/bench_rehearsal_n2.err" || { tail -20 "$OUT/bench_rehearsal_n2.err"; exit 1; }
cat "$OUT/bench_rehearsal_n2.json"
ENET_CRC_AMD_LIB="$ROOT/rusty_enet_amd/lib/variants/libenet_crc_amd_testhooks.so" timeout -k 10 170 \
  python scripts/exp_server_overlap.py > "$OUT/server_overlap.txt" 2>&1 || { tail -20 "$OUT/server_overlap.txt"; exit 1; }
tail -6 "$OUT/server_overlap.txt"
bash scripts/gpu_g1_diff.sh "$TAG/g1diff"
