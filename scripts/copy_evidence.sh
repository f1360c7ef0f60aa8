#!/usr/bin/env bash
# Copy one gpu_r03_final.sh / gpu_profile_round.sh run into a profiles/ directory and
# profiles/pmc_traffic.json (bench.py reads the traffic only while the kernel-source hash
# inside still matches the sources).
#   bash scripts/copy_evidence.sh gpurun_out/<tag> profiles/<round>/final
set -eu
SRC="$1"; DST="$2"
mkdir -p "$DST"
for c in uniform ragged large frag range; do
  cp "$SRC/bench_$c.json" "$DST/"
  cp "$SRC/prof_$c/run_kernel_stats.csv" "$DST/${c}_kernel_stats.csv"
  python3 scripts/pmc_summary.py "$SRC/pmc_$c" > "$DST/${c}_pmc_summary.txt" 2>&1
done
for f in ipc_uniform_summary.txt ipc_ragged_summary.txt ipc_frag_summary.txt rdreq_uniform_summary.txt rdreq_ragged_summary.txt rdreq_frag_summary.txt traffic.json pytest_gpu.log bench_rehearsal_n2.json \
         trace_20_5.json trace_20_5_kernel_trace.csv trace_20_5_vs_line.json trace_200_10.json trace_200_10_kernel_trace.csv \
         trace_200_10_vs_line.json; do
  [ -f "$SRC/$f" ] && cp "$SRC/$f" "$DST/"
done
cp "$SRC/traffic.json" profiles/pmc_traffic.json
