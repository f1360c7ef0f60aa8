#!/usr/bin/env bash
# A/B: whole-line kernel on the LDS-DMA ring (default) vs the same line assignment in a
# register ring with non-temporal loads (linesregs build) vs the line-split register ring
# (nolines build); the linesregs build's uniform parity tests first.
#   gpurun --timeout 900 -- bash scripts/gpu_r03_ab_lines2.sh <tag>
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="${1:-r03_lines2}"
OUT="$ROOT/gpurun_out/$TAG"
mkdir -p "$OUT"
cd "$ROOT"
V=rusty_enet_amd/lib/variants
ENET_CRC_AMD_LIB="$ROOT/$V/libenet_crc_amd_linesregs.so" timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py \
  -m gpu -q -x -k "uniform or full" --timeout 200 --timeout-method thread > "$OUT/pytest_linesregs.log" 2>&1 \
  || { tail -30 "$OUT/pytest_linesregs.log"; exit 1; }
echo "linesregs: $(tail -1 "$OUT/pytest_linesregs.log")"
bash scripts/gpu_ab_configs.sh "$TAG" none "uniform" 4 rusty_enet_amd/lib/libenet_crc_amd.so \
  $V/libenet_crc_amd_linesregs.so $V/libenet_crc_amd_nolines.so
