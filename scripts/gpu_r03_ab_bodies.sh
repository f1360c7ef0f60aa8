#!/usr/bin/env bash
# A/B of the ragged jobs kernel's round bodies (I-cache footprint): generic loop only
# (17.7 KB), + unrolled uniform-top bodies (59 KB), + unrolled mixed bodies (143 KB, the
# default), each build's ragged parity tests first, then ragged/frag bench configs alternating.
#   gpurun --timeout 900 -- bash scripts/gpu_r03_ab_bodies.sh <tag>
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="${1:-r03_bodies}"
OUT="$ROOT/gpurun_out/$TAG"
mkdir -p "$OUT"
cd "$ROOT"
V=rusty_enet_amd/lib/variants
for lib in $V/libenet_crc_amd_bodies0.so $V/libenet_crc_amd_bodies1.so; do
  name=$(basename "$lib" .so)
  ENET_CRC_AMD_LIB="$ROOT/$lib" timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_slot.py \
    -m gpu -q -x --timeout 200 --timeout-method thread \
    > "$OUT/pytest_$name.log" 2>&1 || { tail -30 "$OUT/pytest_$name.log"; exit 1; }
  echo "$name: $(tail -1 "$OUT/pytest_$name.log")"
done
bash scripts/gpu_ab_configs.sh "$TAG" none "ragged frag" 3 rusty_enet_amd/lib/libenet_crc_amd.so \
  $V/libenet_crc_amd_bodies0.so $V/libenet_crc_amd_bodies1.so
