#!/usr/bin/env bash
# Alternating A/B of two builds of the library (ENET_CRC_AMD_LIB) on one bench config:
#   bash scripts/gpu_ab_lib_bench.sh <tag> <config> <libA.so> <libB.so> [reps]
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="$1"; CFG="$2"; A="$3"; B="$4"; REPS="${5:-4}"
OUT="$ROOT/gpurun_out/$TAG"
mkdir -p "$OUT"
cd "$ROOT"
for i in $(seq 1 "$REPS"); do
  for lib in "$A" "$B"; do
    name=$(basename "$lib" .so)
    ENET_CRC_AMD_LIB="$ROOT/$lib" timeout -k 10 200 python bench.py --config "$CFG" --cpu-seconds 0 --no-e2e \
      --no-shard --steps 40 > "$OUT/${name}_$i.json" 2> "$OUT/${name}_$i.err" || exit $?
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['roofline']['kernel_ms'], d['ms_per_step'])" \
      "$OUT/${name}_$i.json" "$name run $i"
  done
done
