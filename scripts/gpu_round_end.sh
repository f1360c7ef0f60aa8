#!/usr/bin/env bash
# End-of-round evidence in one gpurun call: every GPU test, then the profile round
# (bench lines, kernel stats, FETCH_SIZE, counters, traffic.json keyed by the sources).
#   gpurun --timeout 1200 -- bash scripts/gpu_round_end.sh <tag>
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="${1:-end}"
cd "$ROOT"
mkdir -p "gpurun_out/$TAG"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
  > "gpurun_out/$TAG/pytest_gpu.log" 2>&1 || { tail -30 "gpurun_out/$TAG/pytest_gpu.log"; exit 1; }
tail -2 "gpurun_out/$TAG/pytest_gpu.log"
bash scripts/gpu_profile_round.sh "$TAG"
