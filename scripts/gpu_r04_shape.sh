#!/bin/bash
# Round 4: DMA-shape probe (tools/dma_shape) at frag-like and G2-like lengths, then the GPU
# suite on the product (8-lane ragged kernel restored as the default).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-r04_shape}
mkdir -p $O
for args in "1392 1605632 0" "1392 1605632 1" "736 1048576 1" "208 4194304 0"; do
  timeout -k 10 120 tools/dma_shape $args >> $O/dma_shape.txt 2>&1 || { cat $O/dma_shape.txt; exit 1; }
done
cat $O/dma_shape.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -60 $O/pytest_gpu.log; exit 1; }
tail -3 $O/pytest_gpu.log
