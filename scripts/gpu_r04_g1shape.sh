#!/bin/bash
# Round 4: DMA-shape probe on G1's geometry (1M x 1200 B back to back from an aligned base)
# with whole-line pieces (align 128; 256 for the 256-B-piece shapes' line pairs).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-r04_g1shape}
mkdir -p $O
for args in "1200 1048576 0 128" "1200 1048576 0 256" "1200 1048576 0 1"; do
  timeout -k 10 120 tools/dma_shape $args >> $O/dma_shape.txt 2>&1 || { cat $O/dma_shape.txt; exit 1; }
done
cat $O/dma_shape.txt
