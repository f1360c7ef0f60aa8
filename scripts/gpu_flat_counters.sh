#!/usr/bin/env bash
# Counter passes for the ragged config (flat kernels): gpurun -- bash scripts/gpu_flat_counters.sh <tag>
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="${1:-flatc}"
OUT="$ROOT/gpurun_out/$TAG"
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
i=0
for counters in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
                "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
                "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE" \
                "FETCH_SIZE"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --kernel-trace --pmc $counters -d "$OUT/ipc_$i" -o run --output-format csv \
    -- python3 "$ROOT/bench.py" --config ragged --steps 5 --warmup 1 --cpu-seconds 0 --no-verify --no-e2e --no-shard \
    > "$OUT/ipc_$i.log" 2>&1 || exit $?
  echo "[counters] pass $i done" >&2
done
cd "$ROOT"
python3 scripts/pmc_summary.py "$OUT"/ipc_* > "$OUT/summary.txt" 2>&1
cat "$OUT/summary.txt"
