#!/usr/bin/env bash
# Alternating A/B of two builds of the library (ENET_CRC_AMD_LIB) on
# scripts/exp_ragged_overhead.py, in one gpurun call:
#   bash scripts/gpu_ab_lib.sh <tag> <libA.so> <libB.so> [reps]
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="$1"; A="$2"; B="$3"; REPS="${4:-3}"
OUT="$ROOT/gpurun_out/$TAG"
mkdir -p "$OUT"
cd "$ROOT"
for i in $(seq 1 "$REPS"); do
  for lib in "$A" "$B"; do
    name=$(basename "$lib" .so)
    ENET_CRC_AMD_LIB="$ROOT/$lib" timeout -k 10 200 python scripts/exp_ragged_overhead.py --reps 40 \
      > "$OUT/${name}_$i.txt" 2>&1 || exit $?
    echo "== $name run $i"; grep -v amdgpu.ids "$OUT/${name}_$i.txt"
  done
done
