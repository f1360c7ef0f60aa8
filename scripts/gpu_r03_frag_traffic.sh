#!/usr/bin/env bash
# frag_64k (the configs[4] bytes as 49 datagrams per 64 KiB, ragged path): kernel stats and
# FETCH_SIZE / WRITE_SIZE in their own passes.
#   gpurun --timeout 600 -- bash scripts/gpu_r03_frag_traffic.sh <tag>
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="${1:-r03_frag}"
OUT="$ROOT/gpurun_out/$TAG"
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$OUT/prof_frag" -o run --output-format csv \
  -- python3 "$ROOT/bench.py" --config frag --steps 20 --warmup 2 --cpu-seconds 0 --no-verify --no-e2e --no-shard \
  > "$OUT/prof_frag.log" 2>&1 || exit $?
for ctr in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 200 rocprofv3 --kernel-trace --pmc $ctr -d "$OUT/pmc_frag_$ctr" -o run --output-format csv \
    -- python3 "$ROOT/bench.py" --config frag --steps 5 --warmup 1 --cpu-seconds 0 --no-verify --no-e2e --no-shard \
    > "$OUT/pmc_frag_$ctr.log" 2>&1 || exit $?
done
cd "$ROOT"
python3 scripts/pmc_summary.py "$OUT/pmc_frag_FETCH_SIZE" "$OUT/pmc_frag_WRITE_SIZE" > "$OUT/frag_pmc_summary.txt" 2>&1
cat "$OUT/frag_pmc_summary.txt"
