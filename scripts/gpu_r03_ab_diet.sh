#!/usr/bin/env bash
# The ragged jobs kernel's scalar diet (one-instruction division by RJ, round validity and
# job round count carried in the round instead of recomputed): the product build's GPU
# suite, then alternating ragged / frag_64k runs against the previous product (base).
#   gpurun --timeout 900 -- bash scripts/gpu_r03_ab_diet.sh <tag>
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="${1:-r03_diet}"
OUT="$ROOT/gpurun_out/$TAG"
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 300 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread \
  > "$OUT/pytest_gpu.log" 2>&1 || { tail -30 "$OUT/pytest_gpu.log"; exit 1; }
echo "diet: $(tail -1 "$OUT/pytest_gpu.log")"
bash scripts/gpu_ab_configs.sh "$TAG" none "ragged frag" 4 rusty_enet_amd/lib/variants/libenet_crc_amd_base.so \
  rusty_enet_amd/lib/libenet_crc_amd.so
