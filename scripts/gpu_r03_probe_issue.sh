#!/usr/bin/env bash
# Which instruction issue the ragged jobs kernel is sensitive to, and one SALU cut:
#   pv100  +100 dependent VALU per round      pvi100 +100 VALU per round in 4 independent chains
#   ps100  +100 dependent SALU per round      ps300  +300
#   magic  d / RJ as one s_mul_hi instead of hipcc's 11-instruction expansion
# (sources: profiles/r03/parked/claim_merge_and_valu_pad.patch plus the PAD_VALU_INDEP /
# PAD_SALU / RJ_MAGIC blocks of this probe).  The magic build's GPU suite first.
#   gpurun --timeout 900 -- bash scripts/gpu_r03_probe_issue.sh <tag>
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="${1:-r03_pad2}"
OUT="$ROOT/gpurun_out/$TAG"
mkdir -p "$OUT"
cd "$ROOT"
V=rusty_enet_amd/lib/variants
ENET_CRC_AMD_LIB="$ROOT/$V/libenet_crc_amd_magic.so" timeout -k 10 300 python -u -m pytest tests -m gpu -q -x \
  --timeout 200 --timeout-method thread --deselect tests/test_gpu_hooks.py::test_batches_next_to_a_persistent_server \
  > "$OUT/pytest_magic.log" 2>&1 || { tail -30 "$OUT/pytest_magic.log"; exit 1; }
echo "magic: $(tail -1 "$OUT/pytest_magic.log")"
bash scripts/gpu_ab_configs.sh "$TAG" none "ragged" 3 rusty_enet_amd/lib/libenet_crc_amd.so $V/libenet_crc_amd_magic.so \
  $V/libenet_crc_amd_pv100.so $V/libenet_crc_amd_pvi100.so $V/libenet_crc_amd_ps100.so $V/libenet_crc_amd_ps300.so
