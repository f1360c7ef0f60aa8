#!/usr/bin/env bash
# PMC passes (one rocprofv3 run per counter group, kernel-trace only; never combined
# with sys/runtime traces) over a short bench run.  Usage:
#   gpurun --timeout 900 -- bash scripts/gpu_pmc.sh <tag> [config] [extra bench args...]
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="${1:-pmc}"; shift || true
CFG="${1:-uniform}"; shift || true
OUT="$ROOT/gpurun_out/pmc_${CFG}_$TAG"
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
i=0
for counters in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
                "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
                "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE" "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $counters -d "$OUT/pass$i" -o run --output-format csv \
    -- python3 "$ROOT/bench.py" --config "$CFG" --steps 5 --warmup 1 --cpu-seconds 0 --no-verify --no-e2e "$@" \
    > "$OUT/pass$i.log" 2>&1
  rc=$?
  echo "[pmc] pass $i ($counters) rc=$rc" >&2
  if [ $rc -ne 0 ]; then tail -20 "$OUT/pass$i.log" >&2; exit $rc; fi
done
python3 "$ROOT/scripts/pmc_summary.py" "$OUT" > "$OUT/summary.txt" 2>&1; cat "$OUT/summary.txt" >&2
