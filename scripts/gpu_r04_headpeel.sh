#!/bin/bash
# Round 4: whole-line kernel from 16-B aligned bases (head peeled): parity tests, one-process
# timing against base 0, and a kernel trace naming the kernels a base + 16 batch launches.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-r04_headpeel}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 240 --timeout-method thread -k "head_peeled or line_split or whole_lines" > $O/pytest_headpeel.log 2>&1 || { tail -40 $O/pytest_headpeel.log; exit 1; }
tail -1 $O/pytest_headpeel.log
timeout -k 10 300 python -u scripts/exp_headpeel.py > $O/headpeel.txt 2>&1 || { cat $O/headpeel.txt; exit 1; }
grep base $O/headpeel.txt
export TMPDIR=/tmp
(cd /tmp && timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/trace -o run \
  -- python3 $GRAFT_REPO_ROOT/scripts/exp_headpeel.py > $GRAFT_REPO_ROOT/$O/trace.log 2>&1) || exit $?
find $O/trace -name "*kernel_stats.csv" -exec cut -c1-160 {} \; > $O/kernels.txt
cat $O/kernels.txt
