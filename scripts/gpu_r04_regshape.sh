#!/bin/bash
# Round 4: the DMA-shape probe with register-ring shapes next to the LDS-DMA ones (frag-like,
# G2-like and G1-like geometries).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-r04_regshape}
mkdir -p $O
for args in "1392 1605632 0" "740 1048576 0"; do
  timeout -k 10 180 tools/dma_shape $args >> $O/dma_shape.txt 2>&1 || { cat $O/dma_shape.txt; exit 1; }
done
cat $O/dma_shape.txt
