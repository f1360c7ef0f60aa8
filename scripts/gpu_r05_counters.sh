#!/bin/bash
# Instruction / wait counters and read-request sizes of the ragged kernel (G2, frag_64k) on the
# current sources (round 5): same passes as gpu_profile_round.sh, ragged configs only.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/${1:-r05_counters}"
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
for c in ragged frag; do
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum \
    -d "$OUT/rdreq_$c" -o run --output-format csv \
    -- python3 "$ROOT/bench.py" --config $c --steps 5 --warmup 1 --cpu-seconds 0 --no-verify --no-e2e --no-shard \
    > "$OUT/rdreq_$c.log" 2>&1 || exit $?
done
echo "[counters] rdreq done" >&2
i=0
for counters in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
                "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
                "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  for c in ragged frag; do
    timeout -k 10 120 rocprofv3 --kernel-trace --pmc $counters -d "$OUT/ipc_${c}_$i" -o run --output-format csv \
      -- python3 "$ROOT/bench.py" --config $c --steps 5 --warmup 1 --cpu-seconds 0 --no-verify --no-e2e --no-shard \
      > "$OUT/ipc_${c}_$i.log" 2>&1 || exit $?
  done
  echo "[counters] pass $i done" >&2
done
cd "$ROOT"
for c in ragged frag; do
  python3 scripts/pmc_summary.py "$OUT"/ipc_${c}_* > "$OUT/ipc_${c}_summary.txt" 2>&1
  python3 scripts/pmc_summary.py "$OUT/rdreq_$c" > "$OUT/rdreq_${c}_summary.txt" 2>&1
done
echo "[counters] done" >&2
