#!/usr/bin/env bash
# A/B of the ragged jobs kernel's dispatch claim: its own LDS round trip at the loop top
# (default) vs riding in the record read's round trip (cmerge build: make variant NAME=cmerge
# DEFS=-DENET_CRC_CLAIM_MERGE=1); the variant's GPU suite first, then alternating ragged /
# frag_64k runs.
#   gpurun --timeout 900 -- bash scripts/gpu_r03_ab_cmerge.sh <tag>
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="${1:-r03_cmerge}"
OUT="$ROOT/gpurun_out/$TAG"
mkdir -p "$OUT"
cd "$ROOT"
V=rusty_enet_amd/lib/variants
ENET_CRC_AMD_LIB="$ROOT/$V/libenet_crc_amd_cmerge.so" timeout -k 10 300 python -u -m pytest tests -m gpu -q -x \
  --timeout 200 --timeout-method thread --deselect tests/test_gpu_hooks.py::test_batches_next_to_a_persistent_server \
  > "$OUT/pytest_cmerge.log" 2>&1 || { tail -30 "$OUT/pytest_cmerge.log"; exit 1; }
echo "cmerge: $(tail -1 "$OUT/pytest_cmerge.log")"
bash scripts/gpu_ab_configs.sh "$TAG" none "ragged frag" 5 rusty_enet_amd/lib/libenet_crc_amd.so $V/libenet_crc_amd_cmerge.so
