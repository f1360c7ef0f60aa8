#!/bin/bash
# Round 4: the whole-line kernel with its first round's loads issued before the table fill
# (ENET_CRC_EARLY_LOADS): whole-line parity tests on that build, then a same-process A/B on G1
# and the 1392-B MTU batch.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-r04_early}
mkdir -p $O
P=rusty_enet_amd/lib/libenet_crc_amd.so
V=rusty_enet_amd/lib/variants/libenet_crc_amd_early.so
ENET_CRC_AMD_LIB=$GRAFT_REPO_ROOT/$V timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 240 --timeout-method thread > $O/pytest_early.log 2>&1 || { tail -40 $O/pytest_early.log; exit 1; }
tail -1 $O/pytest_early.log
timeout -k 10 300 python -u scripts/ab_ragged.py $V $P --configs g1,mtu --blocks 8 > $O/ab_early.txt 2>&1 || { cat $O/ab_early.txt; exit 1; }
grep -v amdgpu.ids $O/ab_early.txt | grep -v '^{'
