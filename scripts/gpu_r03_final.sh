#!/usr/bin/env bash
# Round-3 final evidence in one call: every GPU test, the N = 2 rehearsal line, then the
# profile round (bench lines, kernel stats, FETCH_SIZE, counters, traffic.json keyed by the
# kernel sources).
#   gpurun --timeout 1200 -- bash scripts/gpu_r03_final.sh <tag>
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="${1:-r03_final}"
OUT="$ROOT/gpurun_out/$TAG"
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
  > "$OUT/pytest_gpu.log" 2>&1 || { tail -30 "$OUT/pytest_gpu.log"; exit 1; }
tail -1 "$OUT/pytest_gpu.log"
BENCH_SHARE_GPUS=1 timeout -k 10 300 python bench.py --gpus 2 --steps 20 --warmup 2 \
  > "$OUT/bench_rehearsal_n2.json" 2> "$OUT/bench_rehearsal_n2.err" || { tail -20 "$OUT/bench_rehearsal_n2.err"; exit 1; }
bash scripts/gpu_profile_round.sh "$TAG"
