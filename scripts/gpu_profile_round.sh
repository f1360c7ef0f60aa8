#!/usr/bin/env bash
# One gpurun call that produces the round's evidence under gpurun_out/<tag>/:
#   bench_<cfg>.json      full bench line per config (uniform also with CPU baseline + end-to-end)
#   prof_<cfg>/           rocprofv3 --kernel-trace --stats of the same bench command
#   pmc_<cfg>/            rocprofv3 --pmc FETCH_SIZE (own pass, kernel trace only)
#   gpurun --timeout 1200 -- bash scripts/gpu_profile_round.sh <tag>
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="${1:-round}"
OUT="$ROOT/gpurun_out/$TAG"
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 600 python bench.py > "$OUT/bench_uniform.json" 2> "$OUT/bench_uniform.err" || exit $?
for c in ragged large; do
  timeout -k 10 300 python bench.py --config $c --cpu-seconds 0 --no-e2e > "$OUT/bench_$c.json" 2> "$OUT/bench_$c.err" || exit $?
done
export TMPDIR=/tmp
cd /tmp
for c in uniform ragged large; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_$c" -o run --output-format csv \
    -- python3 "$ROOT/bench.py" --config $c --steps 20 --warmup 5 --cpu-seconds 0 --no-verify --no-e2e \
    > "$OUT/prof_$c.log" 2>&1 || exit $?
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d "$OUT/pmc_$c" -o run --output-format csv \
    -- python3 "$ROOT/bench.py" --config $c --steps 5 --warmup 1 --cpu-seconds 0 --no-verify --no-e2e \
    > "$OUT/pmc_$c.log" 2>&1 || exit $?
done
echo "[profile] done" >&2
