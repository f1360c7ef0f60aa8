#!/usr/bin/env bash
# Alternating A/B of one environment switch on one bench config, in one process tree:
#   bash scripts/gpu_ab_env.sh <tag> <config> <VAR> <valueA> <valueB> [reps]
# A value "default" leaves VAR unset.  Prints the roofline kernel_ms of each run.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="$1"; CFG="$2"; VAR="$3"; A="$4"; B="$5"; REPS="${6:-4}"
OUT="$ROOT/gpurun_out/$TAG"
mkdir -p "$OUT"
cd "$ROOT"
for i in $(seq 1 "$REPS"); do
  for v in "$A" "$B"; do
    if [ "$v" = default ]; then unset "$VAR"; else export "$VAR=$v"; fi
    timeout -k 10 200 python bench.py --config "$CFG" --cpu-seconds 0 --no-e2e --no-shard --steps 40 \
      > "$OUT/bench_${v}_$i.json" 2> "$OUT/bench_${v}_$i.err" || exit $?
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['roofline']['kernel_ms'], d['ms_per_step'])" \
      "$OUT/bench_${v}_$i.json" "$VAR=$v run $i"
  done
done
unset "$VAR"
