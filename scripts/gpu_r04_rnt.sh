#!/bin/bash
# Round 4: the 8-lane ragged kernel streaming its inner slots non-temporal (ENET_CRC_RAGGED_NT): parity
# suites, then a same-process A/B against the product.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-r04_rnt}
mkdir -p $O
P=rusty_enet_amd/lib/libenet_crc_amd.so
V=rusty_enet_amd/lib/variants/libenet_crc_amd_rnt.so
ENET_CRC_AMD_LIB=$GRAFT_REPO_ROOT/$V timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_slot.py -m gpu -x -v --timeout 240 --timeout-method thread > $O/pytest_gpu_rnt.log 2>&1 || { tail -40 $O/pytest_gpu_rnt.log; exit 1; }
tail -1 $O/pytest_gpu_rnt.log
timeout -k 10 300 python -u scripts/ab_ragged.py $V $P --configs g2,frag,r740,r1396 > $O/ab_rnt.txt 2>&1 || { cat $O/ab_rnt.txt; exit 1; }
grep -v amdgpu.ids $O/ab_rnt.txt | grep -v '^{'
