#!/bin/bash
# Round 4: the 8-lane ragged kernel taking mixed-class rounds in its unrolled bodies (ENET_CRC_SPREAD_FAST): parity
# suites, then a same-process A/B against the product.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-r04_spread}
mkdir -p $O
P=rusty_enet_amd/lib/libenet_crc_amd.so
V=rusty_enet_amd/lib/variants/libenet_crc_amd_spread.so
ENET_CRC_AMD_LIB=$GRAFT_REPO_ROOT/$V timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_slot.py -m gpu -x -v --timeout 240 --timeout-method thread > $O/pytest_gpu_spread.log 2>&1 || { tail -40 $O/pytest_gpu_spread.log; exit 1; }
tail -1 $O/pytest_gpu_spread.log
timeout -k 10 300 python -u scripts/ab_ragged.py $V $P --configs g2,frag,r740,r1396 > $O/ab_spread.txt 2>&1 || { cat $O/ab_spread.txt; exit 1; }
grep -v amdgpu.ids $O/ab_spread.txt | grep -v '^{'
