#!/bin/bash
# Round 4: the 16-packet ragged kernel with 128-B loads and two independent Horner streams
# per lane (ENET_CRC_RAGGED16D): parity suites, then a same-process A/B against the product.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-r04_dual}
mkdir -p $O
P=rusty_enet_amd/lib/libenet_crc_amd.so
D=rusty_enet_amd/lib/variants/libenet_crc_amd_ragged16d.so
ENET_CRC_AMD_LIB=$GRAFT_REPO_ROOT/$D timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_slot.py -m gpu -x -v --timeout 240 --timeout-method thread > $O/pytest_gpu_dual.log 2>&1 || { tail -40 $O/pytest_gpu_dual.log; exit 1; }
tail -1 $O/pytest_gpu_dual.log
timeout -k 10 300 python -u scripts/ab_ragged.py $D $P --configs g2,frag,r740,r1396 > $O/ab_dual.txt 2>&1 || { cat $O/ab_dual.txt; exit 1; }
grep -v amdgpu.ids $O/ab_dual.txt | grep -v '^{'
bash scripts/gpu_r04_g1shape.sh ${1:-r04_dual} || exit $?
