#!/usr/bin/env bash
# A/B of the ragged jobs kernel's chunk geometry: end-aligned 16-B chunks (default; a chunk
# may straddle two lines) vs whole lines (rlines build: make variant NAME=rlines
# DEFS=-DENET_CRC_RAGGED_LINES=1): the variant's whole GPU suite first, then alternating
# ragged / frag_64k runs (also rlinesnt: inner lines by non-temporal DMAs,
# -DENET_CRC_RAGGED_LINES_NT=1), then the line form's FETCH_SIZE on the ragged config.
#   gpurun --timeout 1200 -- bash scripts/gpu_r03_ab_rlines.sh <tag>
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="${1:-r03_rlines}"
OUT="$ROOT/gpurun_out/$TAG"
mkdir -p "$OUT"
cd "$ROOT"
V=rusty_enet_amd/lib/variants
for n in rlines rlinesnt; do
  ENET_CRC_AMD_LIB="$ROOT/$V/libenet_crc_amd_$n.so" timeout -k 10 300 python -u -m pytest tests -m gpu -q -x \
    --timeout 200 --timeout-method thread --deselect tests/test_gpu_hooks.py::test_batches_next_to_a_persistent_server \
    > "$OUT/pytest_$n.log" 2>&1 || { tail -30 "$OUT/pytest_$n.log"; exit 1; }
  echo "$n: $(tail -1 "$OUT/pytest_$n.log")"
done
bash scripts/gpu_ab_configs.sh "$TAG" none "ragged frag" 4 rusty_enet_amd/lib/libenet_crc_amd.so $V/libenet_crc_amd_rlines.so \
  $V/libenet_crc_amd_rlinesnt.so || exit $?
export TMPDIR=/tmp
cd /tmp
ENET_CRC_AMD_LIB="$ROOT/$V/libenet_crc_amd_rlines.so" timeout -k 10 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE \
  -d "$OUT/pmc_rlines" -o run --output-format csv -- python3 "$ROOT/bench.py" --config ragged --steps 5 --warmup 1 \
  --cpu-seconds 0 --no-verify --no-e2e --no-shard > "$OUT/pmc_rlines.log" 2>&1 || exit $?
cd "$ROOT"
python3 scripts/pmc_summary.py "$OUT/pmc_rlines" > "$OUT/pmc_rlines_summary.txt" 2>&1
cat "$OUT/pmc_rlines_summary.txt"
