#!/usr/bin/env bash
# A/B of the register-ring whole-line kernel's issue order: default, first round's loads
# before the LDS table fill (early), and additionally each slot's next-round load before its
# lookups (earlyfirst); each variant's uniform parity tests first.
#   gpurun --timeout 900 -- bash scripts/gpu_r03_ab_lines4.sh <tag>
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="${1:-r03_lines4}"
OUT="$ROOT/gpurun_out/$TAG"
mkdir -p "$OUT"
cd "$ROOT"
V=rusty_enet_amd/lib/variants
for name in early earlyfirst; do
  ENET_CRC_AMD_LIB="$ROOT/$V/libenet_crc_amd_$name.so" timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py \
    -m gpu -q -x -k "uniform or full" --timeout 200 --timeout-method thread > "$OUT/pytest_$name.log" 2>&1 \
    || { tail -30 "$OUT/pytest_$name.log"; exit 1; }
  echo "$name: $(tail -1 "$OUT/pytest_$name.log")"
done
bash scripts/gpu_ab_configs.sh "$TAG" none "uniform" 4 rusty_enet_amd/lib/libenet_crc_amd.so \
  $V/libenet_crc_amd_early.so $V/libenet_crc_amd_earlyfirst.so
