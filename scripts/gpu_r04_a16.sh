#!/bin/bash
# Round 4: the 8-lane ragged kernel with 16-B-aligned chunks (ENET_CRC_RAGGED_A16) and with
# a 2-slot ring as well (a16r2): parity suites of both, then same-process A/Bs against the
# product on G2, frag_64k and uniform-length batches through the ragged entry; the DMA-shape
# probe's wider pieces.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-r04_a16}
mkdir -p $O
P=rusty_enet_amd/lib/libenet_crc_amd.so
V=rusty_enet_amd/lib/variants
for v in a16 a16r2; do
  ENET_CRC_AMD_LIB=$GRAFT_REPO_ROOT/$V/libenet_crc_amd_$v.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_slot.py -m gpu -x -v --timeout 240 --timeout-method thread > $O/pytest_gpu_$v.log 2>&1 || { tail -40 $O/pytest_gpu_$v.log; exit 1; }
  tail -1 $O/pytest_gpu_$v.log
done
for v in a16 a16r2; do
  timeout -k 10 300 python -u scripts/ab_ragged.py $V/libenet_crc_amd_$v.so $P --configs g2,frag,r740,r1396 > $O/ab_$v.txt 2>&1 || { cat $O/ab_$v.txt; exit 1; }
  grep -v amdgpu.ids $O/ab_$v.txt | grep -v '^{'
done
for args in "1392 1605632 0" "740 1048576 0 16"; do
  timeout -k 10 120 tools/dma_shape $args >> $O/dma_shape.txt 2>&1 || { cat $O/dma_shape.txt; exit 1; }
done
cat $O/dma_shape.txt
