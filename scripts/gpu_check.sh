#!/usr/bin/env bash
# One gpurun call: GPU parity tests, a bench line, and a rocprofv3 kernel-trace
# summary.  Each GPU step has its own time limit; a fault/abort/timeout ends the
# script (no further GPU work), a plain test failure (pytest exit 1) does not.
#   gpurun --timeout 1200 -- bash scripts/gpu_check.sh [tag] [bench-config]
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="${1:-r01}"
CFG="${2:-uniform}"
OUT="$ROOT/gpurun_out"
mkdir -p "$OUT"
cd "$ROOT"

fatal() {  # exit codes that mean the GPU step died: stop here
  case "$1" in 0|1) return 1 ;; *) return 0 ;; esac
}

echo "[gpu_check] pytest -m gpu" >&2
timeout -k 10 900 python -m pytest tests -m gpu -x -q > "$OUT/pytest_gpu_$TAG.log" 2>&1
rc=$?
echo "[gpu_check] pytest rc=$rc" >&2
tail -5 "$OUT/pytest_gpu_$TAG.log" >&2
if fatal $rc; then echo "[gpu_check] stopping after pytest rc=$rc" >&2; exit $rc; fi

echo "[gpu_check] bench $CFG" >&2
timeout -k 10 400 python bench.py --config "$CFG" > "$OUT/bench_${CFG}_$TAG.json" 2> "$OUT/bench_${CFG}_$TAG.err"
brc=$?
cat "$OUT/bench_${CFG}_$TAG.json" >&2
if [ $brc -ne 0 ]; then tail -20 "$OUT/bench_${CFG}_$TAG.err" >&2; exit $brc; fi

echo "[gpu_check] rocprofv3 kernel trace" >&2
export TMPDIR=/tmp
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/prof_${CFG}_$TAG" -o run --output-format csv \
  -- python3 "$ROOT/bench.py" --config "$CFG" --steps 20 --warmup 5 --cpu-seconds 0 --no-verify --no-e2e \
  > "$OUT/prof_${CFG}_$TAG.log" 2>&1
prc=$?
echo "[gpu_check] rocprof rc=$prc" >&2
find "$OUT/prof_${CFG}_$TAG" -name '*stats*' -exec cat {} \; >&2 2>/dev/null | head -20
exit $(( rc != 0 ? rc : prc ))
