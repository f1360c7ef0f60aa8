#!/usr/bin/env bash
# A/B of the wave-per-packet kernel: LDS-DMA ring (default) vs register ring with
# non-temporal loads (waveregs build); the variant's long-packet parity tests first.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="${1:-r03_waveregs}"
OUT="$ROOT/gpurun_out/$TAG"
mkdir -p "$OUT"
cd "$ROOT"
V=rusty_enet_amd/lib/variants
ENET_CRC_AMD_LIB="$ROOT/$V/libenet_crc_amd_waveregs.so" timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py \
  -m gpu -q -x -k "long or large or 64k" --timeout 200 --timeout-method thread > "$OUT/pytest_waveregs.log" 2>&1 \
  || { tail -30 "$OUT/pytest_waveregs.log"; exit 1; }
echo "waveregs: $(tail -1 "$OUT/pytest_waveregs.log")"
bash scripts/gpu_ab_configs.sh "$TAG" none "large" 4 rusty_enet_amd/lib/libenet_crc_amd.so $V/libenet_crc_amd_waveregs.so
