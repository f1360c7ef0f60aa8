#!/usr/bin/env bash
# A/B: ragged jobs kernel with plain DMAs (default) vs non-temporal DMAs for the inner pieces
# of the fast rounds (raggednt build), after the variant's parity tests and the server tests.
#   gpurun --timeout 900 -- bash scripts/gpu_r03_ab_raggednt.sh <tag>
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="${1:-r03_raggednt}"
OUT="$ROOT/gpurun_out/$TAG"
mkdir -p "$OUT"
cd "$ROOT"
V=rusty_enet_amd/lib/variants
timeout -k 10 300 python -u -m pytest tests/test_gpu_hooks.py -m gpu -q -x --timeout 200 --timeout-method thread \
  > "$OUT/pytest_hooks.log" 2>&1 || { tail -30 "$OUT/pytest_hooks.log"; exit 1; }
echo "hooks: $(tail -1 "$OUT/pytest_hooks.log")"
ENET_CRC_AMD_LIB="$ROOT/$V/libenet_crc_amd_raggednt.so" timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py \
  tests/test_gpu_slot.py -m gpu -q -x --timeout 200 --timeout-method thread > "$OUT/pytest_raggednt.log" 2>&1 \
  || { tail -30 "$OUT/pytest_raggednt.log"; exit 1; }
echo "raggednt: $(tail -1 "$OUT/pytest_raggednt.log")"
bash scripts/gpu_ab_configs.sh "$TAG" none "ragged frag" 3 rusty_enet_amd/lib/libenet_crc_amd.so \
  $V/libenet_crc_amd_raggednt.so
