#!/usr/bin/env bash
# Alternating runs of several values of one environment switch on one bench config:
#   bash scripts/gpu_ab_env_multi.sh <tag> <config> <VAR> <reps> <value>...   ("default" = unset)
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="$1"; CFG="$2"; VAR="$3"; REPS="$4"; shift 4
OUT="$ROOT/gpurun_out/$TAG"
mkdir -p "$OUT"
cd "$ROOT"
for i in $(seq 1 "$REPS"); do
  for v in "$@"; do
    if [ "$v" = default ]; then unset "$VAR"; else export "$VAR=$v"; fi
    timeout -k 10 200 python bench.py --config "$CFG" --cpu-seconds 0 --no-e2e --no-shard --steps 40 \
      > "$OUT/bench_${v}_$i.json" 2> "$OUT/bench_${v}_$i.err" || exit $?
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['roofline']['kernel_ms'], d['ms_per_step'])" \
      "$OUT/bench_${v}_$i.json" "$VAR=$v run $i"
  done
done
