#!/usr/bin/env bash
# A/B of the whole-line kernel's combine: default (3-level replicated tree, select after the
# handover step) vs the per-lane shift block (one lookup round + DPP XOR) with the handover
# step masked to the lanes that need it (shift build); the variant's uniform parity first.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="${1:-r03_shift}"
OUT="$ROOT/gpurun_out/$TAG"
mkdir -p "$OUT"
cd "$ROOT"
V=rusty_enet_amd/lib/variants
ENET_CRC_AMD_LIB="$ROOT/$V/libenet_crc_amd_shift.so" timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py \
  -m gpu -q -x -k "uniform or full" --timeout 200 --timeout-method thread > "$OUT/pytest_shift.log" 2>&1 \
  || { tail -30 "$OUT/pytest_shift.log"; exit 1; }
echo "shift: $(tail -1 "$OUT/pytest_shift.log")"
bash scripts/gpu_ab_configs.sh "$TAG" none "uniform" 5 rusty_enet_amd/lib/libenet_crc_amd.so $V/libenet_crc_amd_shift.so
