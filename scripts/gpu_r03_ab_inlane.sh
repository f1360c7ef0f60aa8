#!/usr/bin/env bash
# A/B of the ragged jobs kernel's in-lane combine: two trips with an unreplicated M32^2
# (default) vs three conflict-free trips (inlane3 build); the variant's ragged parity first,
# then its bank-conflict counters.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="${1:-r03_inlane}"
OUT="$ROOT/gpurun_out/$TAG"
mkdir -p "$OUT"
cd "$ROOT"
V=rusty_enet_amd/lib/variants
ENET_CRC_AMD_LIB="$ROOT/$V/libenet_crc_amd_inlane3.so" timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py \
  tests/test_gpu_slot.py -m gpu -q -x --timeout 200 --timeout-method thread > "$OUT/pytest_inlane3.log" 2>&1 \
  || { tail -30 "$OUT/pytest_inlane3.log"; exit 1; }
echo "inlane3: $(tail -1 "$OUT/pytest_inlane3.log")"
bash scripts/gpu_ab_configs.sh "$TAG" none "ragged frag" 4 rusty_enet_amd/lib/libenet_crc_amd.so $V/libenet_crc_amd_inlane3.so || exit $?
export TMPDIR=/tmp
cd /tmp
ENET_CRC_AMD_LIB="$ROOT/$V/libenet_crc_amd_inlane3.so" timeout -k 10 120 rocprofv3 --kernel-trace --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE \
  -d "$OUT/ipc_inlane3" -o run --output-format csv -- python3 "$ROOT/bench.py" --config ragged --steps 5 --warmup 1 \
  --cpu-seconds 0 --no-verify --no-e2e --no-shard > "$OUT/ipc_inlane3.log" 2>&1 || exit $?
cd "$ROOT"
python3 scripts/pmc_summary.py "$OUT/ipc_inlane3" > "$OUT/ipc_inlane3_summary.txt" 2>&1
cat "$OUT/ipc_inlane3_summary.txt"
