#!/usr/bin/env bash
# Ragged-path counters for one library build (ENET_CRC_AMD_LIB): FETCH_SIZE / WRITE_SIZE
# and the instruction / wait counters, each pass on its own, kernel trace only.
#   bash scripts/gpu_ragged_counters.sh <tag> <lib.so> [config]
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="$1"; LIB="$2"; CFG="${3:-ragged}"
OUT="$ROOT/gpurun_out/$TAG"
mkdir -p "$OUT"
export TMPDIR=/tmp
export ENET_CRC_AMD_LIB="$ROOT/$LIB"
cd /tmp
i=0
for counters in "FETCH_SIZE" "WRITE_SIZE" \
                "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
                "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
                "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --kernel-trace --pmc $counters -d "$OUT/c_$i" -o run --output-format csv \
    -- python3 "$ROOT/bench.py" --config "$CFG" --steps 5 --warmup 1 --cpu-seconds 0 --no-verify --no-e2e --no-shard \
    > "$OUT/c_$i.log" 2>&1 || exit $?
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$OUT/stats" -o run --output-format csv \
  -- python3 "$ROOT/bench.py" --config "$CFG" --steps 20 --warmup 2 --cpu-seconds 0 --no-verify --no-e2e --no-shard \
  > "$OUT/stats.log" 2>&1 || exit $?
cd "$ROOT"
python3 scripts/pmc_summary.py "$OUT"/c_* > "$OUT/summary.txt" 2>&1
find "$OUT/stats" -name '*kernel_stats*' -exec cp {} "$OUT/kernel_stats.csv" \;
cat "$OUT/summary.txt"
