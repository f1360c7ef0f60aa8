#!/bin/bash
# Round 4: the 8-lane ragged kernel with a 2-slot ring (ENET_CRC_RAGGED_RING=2 build; the
# DMA-shape probe streams 3-4 % faster at ring 2 than 3): parity suites, then a
# same-process A/B against the product (ring 3) on G2 and frag_64k.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-r04_ring2}
mkdir -p $O
P=rusty_enet_amd/lib/libenet_crc_amd.so
V=rusty_enet_amd/lib/variants/libenet_crc_amd_ring2.so
ENET_CRC_AMD_LIB=$GRAFT_REPO_ROOT/$V timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_slot.py -m gpu -x -v --timeout 240 --timeout-method thread > $O/pytest_gpu_ring2.log 2>&1 || { tail -40 $O/pytest_gpu_ring2.log; exit 1; }
tail -2 $O/pytest_gpu_ring2.log
timeout -k 10 200 python -u scripts/ab_ragged.py $V $P --configs g2,frag > $O/ab_ring2.txt 2>&1 || { cat $O/ab_ring2.txt; exit 1; }
grep -v amdgpu.ids $O/ab_ring2.txt | grep -v '^{'
bash scripts/gpu_r04_a16.sh ${1:-r04_ring2} || exit $?
