#!/usr/bin/env bash
# One gpurun call: full GPU test suite, the default bench line, the range-coder bench
# line and a rocprofv3 kernel-trace summary of the range bench.  Each GPU step has its
# own time limit; a fault/abort/timeout ends the script.
#   gpurun --timeout 1200 -- bash scripts/gpu_range_round.sh <tag>
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="${1:-r01}"
OUT="$ROOT/gpurun_out"
mkdir -p "$OUT"
cd "$ROOT"
step() {  # step <seconds> <log> <cmd...>
  local t="$1" log="$2"; shift 2
  echo "[round] $*" >&2
  timeout -k 10 "$t" "$@" > "$log" 2>&1
  local rc=$?
  echo "[round] rc=$rc" >&2
  tail -4 "$log" >&2
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
  if grep -q "HSA_STATUS_ERROR\|Memory access fault" "$log"; then exit 99; fi
  return $rc
}
step 600 "$OUT/pytest_gpu_$TAG.log" python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread
step 300 "$OUT/bench_uniform_$TAG.json" python bench.py
step 300 "$OUT/bench_range_$TAG.json" python bench.py --config range
export TMPDIR=/tmp
cd /tmp
step 300 "$OUT/prof_range_$TAG.log" rocprofv3 --kernel-trace --stats -d "$OUT/prof_range_$TAG" -o run --output-format csv \
  -- python3 "$ROOT/bench.py" --config range --steps 3 --warmup 1 --cpu-seconds 0 --no-verify
find "$OUT/prof_range_$TAG" -name '*kernel_stats*' -exec cat {} \; >&2
