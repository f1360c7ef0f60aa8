#!/bin/bash
# Round 4: G1 launch-time dynamics within one process, and the same-buffer read ceiling.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r04_ramp
mkdir -p $O
timeout -k 10 240 python -u scripts/exp_clock_ramp.py > $O/ramp.txt 2>&1 || exit $?
timeout -k 10 240 python -u bench.py --steps 20 --warmup 5 --no-e2e --cpu-seconds 1 > $O/bench_20_5.json 2> $O/bench_20_5.err || exit $?
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 5 --no-e2e --cpu-seconds 1 --no-shard > $GRAFT_REPO_ROOT/$O/bench_prof.json 2> $GRAFT_REPO_ROOT/$O/bench_prof.err
