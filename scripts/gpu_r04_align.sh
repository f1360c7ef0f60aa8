#!/bin/bash
# Round 4: DMA-shape probe on 4-B-aligned (not 16-B) lane loads, as arbitrary datagram
# lengths give the ragged kernels, against the same pattern rounded to 16-B boundaries;
# the profiler's counter list (for a 64-B / 128-B read request split).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-r04_align}
mkdir -p $O
for args in "1396 1605632 0" "1396 1605632 0 16" "740 1048576 0" "740 1048576 0 16" "1392 1605632 0"; do
  timeout -k 10 120 tools/dma_shape $args >> $O/dma_shape.txt 2>&1 || { cat $O/dma_shape.txt; exit 1; }
done
cat $O/dma_shape.txt
(cd /tmp && timeout -s KILL 60 rocprofv3 -L > $GRAFT_REPO_ROOT/$O/counters.txt 2>&1) || true
grep -o "TCC_EA0_RD[A-Z0-9_]*\|TCC_BUBBLE[A-Z0-9_]*\|TCC_REQ[A-Z0-9_]*" $O/counters.txt | sort -u | head -40 || true
