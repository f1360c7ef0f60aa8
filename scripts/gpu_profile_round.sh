#!/usr/bin/env bash
# One gpurun call that produces the round's roofline evidence under gpurun_out/<tag>/:
#   bench_<cfg>.json   the bench line per config (uniform also with CPU baseline + end-to-end)
#   prof_<cfg>/        rocprofv3 --kernel-trace --stats of the same bench command
#   pmc_<cfg>/         rocprofv3 --pmc FETCH_SIZE (own pass, kernel trace only)
#   ipc_<cfg>_<n>/     instruction / cycle counters (own passes) for uniform and ragged
#   traffic.json       scripts/traffic_summary.py over the above (kernel-source hash inside)
#   gpurun --timeout 1200 -- bash scripts/gpu_profile_round.sh <tag>
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="${1:-round}"
OUT="$ROOT/gpurun_out/$TAG"
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 300 python bench.py > "$OUT/bench_uniform.json" 2> "$OUT/bench_uniform.err" || exit $?
echo "[profile] uniform bench done" >&2
for c in ragged large frag; do
  timeout -k 10 200 python bench.py --config $c --cpu-seconds 0 --no-e2e > "$OUT/bench_$c.json" 2> "$OUT/bench_$c.err" || exit $?
  echo "[profile] $c bench done" >&2
done
timeout -k 10 300 python bench.py --config range > "$OUT/bench_range.json" 2> "$OUT/bench_range.err" || exit $?
echo "[profile] range bench done" >&2
export TMPDIR=/tmp
cd /tmp
for c in uniform ragged large frag range; do
  steps=20; [ $c = range ] && steps=3
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_$c" -o run --output-format csv \
    -- python3 "$ROOT/bench.py" --config $c --steps $steps --warmup 2 --cpu-seconds 0 --no-verify --no-e2e --no-shard \
    > "$OUT/prof_$c.log" 2>&1 || exit $?
  echo "[profile] $c kernel stats done" >&2
done
for c in uniform ragged large frag; do
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d "$OUT/pmc_$c" -o run --output-format csv \
    -- python3 "$ROOT/bench.py" --config $c --steps 5 --warmup 1 --cpu-seconds 0 --no-verify --no-e2e --no-shard \
    > "$OUT/pmc_$c.log" 2>&1 || exit $?
  echo "[profile] $c FETCH_SIZE done" >&2
done
timeout -k 10 300 rocprofv3 --kernel-trace --pmc TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum -d "$OUT/pmc_range" -o run --output-format csv \
  -- python3 "$ROOT/bench.py" --config range --steps 2 --warmup 1 --cpu-seconds 0 --no-verify \
  > "$OUT/pmc_range.log" 2>&1 || exit $?
echo "[profile] range read requests done" >&2
# L2-to-memory read requests by size (is FETCH_SIZE x 2 right for the ragged kernel's partial lines?)
for c in uniform ragged frag; do
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum \
    -d "$OUT/rdreq_$c" -o run --output-format csv \
    -- python3 "$ROOT/bench.py" --config $c --steps 5 --warmup 1 --cpu-seconds 0 --no-verify --no-e2e --no-shard \
    > "$OUT/rdreq_$c.log" 2>&1 || exit $?
done
echo "[profile] read request sizes done" >&2
i=0
for counters in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
                "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
                "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  for c in uniform ragged frag; do
    timeout -k 10 120 rocprofv3 --kernel-trace --pmc $counters -d "$OUT/ipc_${c}_$i" -o run --output-format csv \
      -- python3 "$ROOT/bench.py" --config $c --steps 5 --warmup 1 --cpu-seconds 0 --no-verify --no-e2e --no-shard \
      > "$OUT/ipc_${c}_$i.log" 2>&1 || exit $?
  done
  echo "[profile] counter pass $i done" >&2
done
cd "$ROOT"
python3 scripts/traffic_summary.py "gpurun_out/$TAG" > "$OUT/traffic.json" 2>&1 || exit $?
for c in uniform ragged frag; do
  python3 scripts/pmc_summary.py "$OUT"/ipc_${c}_* > "$OUT/ipc_${c}_summary.txt" 2>&1
  python3 scripts/pmc_summary.py "$OUT/rdreq_$c" > "$OUT/rdreq_${c}_summary.txt" 2>&1
done
# One bench process's per-launch kernel trace, the driver's command shape and the default
# (the launch-time series behind the line).
for spec in "20 5" "200 10"; do
  set -- $spec
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/trace_$1_$2" -o run \
    -- python3 "$ROOT/bench.py" --steps $1 --warmup $2 --cpu-seconds 0 --no-e2e --no-shard > "$OUT/trace_$1_$2.json" 2> "$OUT/trace_$1_$2.err") || exit $?
  python3 scripts/trace_vs_line.py "$OUT/trace_$1_$2" "$OUT/trace_$1_$2.json" --csv "$OUT/trace_$1_$2_kernel_trace.csv" \
    > "$OUT/trace_$1_$2_vs_line.json" 2>&1
done
echo "[profile] launch traces done" >&2
echo "[profile] done" >&2
