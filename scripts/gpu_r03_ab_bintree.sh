#!/usr/bin/env bash
# A/B of the ragged jobs kernel's cross-lane combine: radix-4 tree (default at commit
# c593fe8) vs the 3-level binary tree (bintree build: make variant NAME=bintree
# DEFS=-DENET_CRC_JOBS_BINTREE=1 on that commit; the binary tree is the default since);
# the variant's ragged parity first, then its bank-conflict counters.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="${1:-r03_bintree}"
OUT="$ROOT/gpurun_out/$TAG"
mkdir -p "$OUT"
cd "$ROOT"
V=rusty_enet_amd/lib/variants
ENET_CRC_AMD_LIB="$ROOT/$V/libenet_crc_amd_bintree.so" timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py \
  tests/test_gpu_slot.py -m gpu -q -x --timeout 200 --timeout-method thread > "$OUT/pytest_bintree.log" 2>&1 \
  || { tail -30 "$OUT/pytest_bintree.log"; exit 1; }
echo "bintree: $(tail -1 "$OUT/pytest_bintree.log")"
bash scripts/gpu_ab_configs.sh "$TAG" none "ragged frag" 4 rusty_enet_amd/lib/libenet_crc_amd.so $V/libenet_crc_amd_bintree.so || exit $?
export TMPDIR=/tmp
cd /tmp
ENET_CRC_AMD_LIB="$ROOT/$V/libenet_crc_amd_bintree.so" timeout -k 10 120 rocprofv3 --kernel-trace --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE \
  -d "$OUT/ipc_bintree" -o run --output-format csv -- python3 "$ROOT/bench.py" --config ragged --steps 5 --warmup 1 \
  --cpu-seconds 0 --no-verify --no-e2e --no-shard > "$OUT/ipc_bintree.log" 2>&1 || exit $?
cd "$ROOT"
python3 scripts/pmc_summary.py "$OUT/ipc_bintree" > "$OUT/ipc_bintree_summary.txt" 2>&1
cat "$OUT/ipc_bintree_summary.txt"
