#!/bin/bash
# Round 4: per-launch kernel times of the ragged kernel in one bench process (G2, 300 timed
# launches after 5 warmup): how long does it take to reach its steady rate?
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-r04_rramp}
mkdir -p $O
export TMPDIR=/tmp
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$O/trace_ragged -o run \
  -- python3 $GRAFT_REPO_ROOT/bench.py --config ragged --steps 300 --warmup 5 --cpu-seconds 0 --no-e2e --no-shard \
  > $GRAFT_REPO_ROOT/$O/trace_ragged.json 2> $GRAFT_REPO_ROOT/$O/trace_ragged.err) || exit $?
python3 scripts/launch_series.py $O/trace_ragged --kernel crc32_ragged_jobs_kernel > $O/ragged_series.txt 2>&1 || true
cat $O/ragged_series.txt
