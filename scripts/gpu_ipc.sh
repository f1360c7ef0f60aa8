#!/usr/bin/env bash
# Instruction / wait counters (three --pmc passes) for one bench config:
#   bash scripts/gpu_ipc.sh <tag> <config>
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="${1:-ipc}"; CFG="${2:-ragged}"
OUT="$ROOT/gpurun_out/$TAG"
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
i=0
for counters in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
                "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
                "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --kernel-trace --pmc $counters -d "$OUT/ipc_$i" -o run --output-format csv \
    -- python3 "$ROOT/bench.py" --config "$CFG" --steps 5 --warmup 1 --cpu-seconds 0 --no-verify --no-e2e --no-shard \
    > "$OUT/ipc_$i.log" 2>&1 || exit $?
done
cd "$ROOT"
python3 scripts/pmc_summary.py "$OUT"/ipc_* > "$OUT/ipc_summary.txt" 2>&1
cat "$OUT/ipc_summary.txt"
