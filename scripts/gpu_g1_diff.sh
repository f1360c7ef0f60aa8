#!/usr/bin/env bash
# G1 ceiling evidence: the read probe P9 (every line of a round read
# once, whole, non-temporal, the kernel's 16 lookups per slot) against the G1 kernel,
# under the same counters, in one call.  tools/dma_probe must be built (make probes).
#   gpurun -- bash scripts/gpu_g1_diff.sh <tag>
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="${1:-g1diff}"
OUT="$ROOT/gpurun_out/$TAG"
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
PROBE="$ROOT/tools/dma_probe"
timeout -k 10 120 env PROBE_SHARED=1 PROBE_RANDOM=1 "$PROBE" > "$OUT/probe_times.txt" 2>&1 || exit $?
cat "$OUT/probe_times.txt"
timeout -k 10 200 env PROBE_SHARED=1 PROBE_RANDOM=1 rocprofv3 --kernel-trace --stats -d "$OUT/stats_probe" -o run \
  --output-format csv -- "$PROBE" > "$OUT/stats_probe.log" 2>&1 || exit $?
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$OUT/stats_bench" -o run --output-format csv \
  -- python3 "$ROOT/bench.py" --config uniform --steps 20 --warmup 2 --cpu-seconds 0 --no-verify --no-e2e --no-shard \
  > "$OUT/stats_bench.log" 2>&1 || exit $?
i=0
for counters in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
                "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
                "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE" \
                "FETCH_SIZE"; do
  i=$((i+1))
  timeout -k 10 120 env PROBE_SHARED=1 PROBE_RANDOM=1 rocprofv3 --kernel-trace --pmc $counters -d "$OUT/probe_$i" \
    -o run --output-format csv -- "$PROBE" > "$OUT/probe_$i.log" 2>&1 || exit $?
  timeout -k 10 120 rocprofv3 --kernel-trace --pmc $counters -d "$OUT/bench_$i" -o run --output-format csv \
    -- python3 "$ROOT/bench.py" --config uniform --steps 5 --warmup 1 --cpu-seconds 0 --no-verify --no-e2e --no-shard \
    > "$OUT/bench_$i.log" 2>&1 || exit $?
  echo "[g1diff] pass $i done" >&2
done
cd "$ROOT"
PMC_FILTER=probe python3 scripts/pmc_summary.py "$OUT"/probe_[0-9]* > "$OUT/probe_summary.txt" 2>&1
python3 scripts/pmc_summary.py "$OUT"/bench_[0-9]* > "$OUT/bench_summary.txt" 2>&1
cat "$OUT/probe_summary.txt" "$OUT/bench_summary.txt"
