#!/bin/bash
# Round 4: DMA-shape probe, then the 16-packet / 128-B-load ragged kernel (gpu_r04_w.sh),
# then the GPU suite on the product.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-r04_sw}
mkdir -p $O
for args in "1392 1605632 0" "1392 1605632 1" "736 1048576 1" "208 4194304 0"; do
  timeout -k 10 120 tools/dma_shape $args >> $O/dma_shape.txt 2>&1 || { cat $O/dma_shape.txt; exit 1; }
done
cat $O/dma_shape.txt
bash scripts/gpu_r04_w.sh ${1:-r04_sw} || exit $?
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -60 $O/pytest_gpu.log; exit 1; }
tail -3 $O/pytest_gpu.log
