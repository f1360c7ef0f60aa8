#!/usr/bin/env bash
# Kernel stats and inter-kernel gaps (rocprofv3 --kernel-trace --stats) for two values
# of one environment switch on one case of scripts/exp_ragged_overhead.py:
#   bash scripts/gpu_ab_env_prof.sh <tag> <VAR> <valueA> <valueB> <case> [reps]
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="$1"; VAR="$2"; A="$3"; B="$4"; CASE="$5"; REPS="${6:-2}"
OUT="$ROOT/gpurun_out/$TAG"
mkdir -p "$OUT"
export TMPDIR=/tmp
for i in $(seq 1 "$REPS"); do
  for v in "$A" "$B"; do
    if [ "$v" = default ]; then unset "$VAR"; else export "$VAR=$v"; fi
    d="$OUT/${v}_$i"
    timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$d" -o run --output-format csv \
      -- python3 "$ROOT/scripts/exp_ragged_overhead.py" --reps 40 --only "$CASE" > "$d.log" 2>&1 || exit $?
    echo "== $VAR=$v run $i"; grep " us " "$d.log"
    python3 "$ROOT/scripts/trace_gaps.py" "$d"
  done
done
unset "$VAR"
