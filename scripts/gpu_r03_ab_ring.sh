#!/usr/bin/env bash
# A/B of the ragged jobs kernel's LDS split: DMA ring 3 + 8 job slots (default), ring 4 +
# 4 job slots (r4s4), ring 3 + 4 job slots (r3s4); each variant's ragged parity first.
#   gpurun --timeout 900 -- bash scripts/gpu_r03_ab_ring.sh <tag>
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="${1:-r03_ring}"
OUT="$ROOT/gpurun_out/$TAG"
mkdir -p "$OUT"
cd "$ROOT"
V=rusty_enet_amd/lib/variants
for name in r4s4 r3s4; do
  ENET_CRC_AMD_LIB="$ROOT/$V/libenet_crc_amd_$name.so" timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py \
    tests/test_gpu_slot.py -m gpu -q -x --timeout 200 --timeout-method thread > "$OUT/pytest_$name.log" 2>&1 \
    || { tail -30 "$OUT/pytest_$name.log"; exit 1; }
  echo "$name: $(tail -1 "$OUT/pytest_$name.log")"
done
bash scripts/gpu_ab_configs.sh "$TAG" none "ragged frag" 3 rusty_enet_amd/lib/libenet_crc_amd.so \
  $V/libenet_crc_amd_r4s4.so $V/libenet_crc_amd_r3s4.so
