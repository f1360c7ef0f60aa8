#!/bin/bash
# A variant build through the ragged GPU parity tests (ENET_CRC_AMD_LIB), then the same-process
# A/B against the product.   gpurun -- bash scripts/gpu_r05_variant.sh <tag> <variant> [configs] [blocks] [pytest -k]
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/$1
V=$2
CFG=${3:-g2,frag,r740}
BLK=${4:-8}
K=${5:-ragged or frag or every_length or golden or host or ring or slot or full_size}
mkdir -p $O
ENET_CRC_AMD_LIB=$PWD/rusty_enet_amd/lib/variants/libenet_crc_amd_$V.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_slot.py tests/test_gpu_ring.py -m gpu -x -q --timeout 240 --timeout-method thread -k "$K" > $O/pytest_$V.log 2>&1 || { tail -40 $O/pytest_$V.log; exit 1; }
tail -2 $O/pytest_$V.log
timeout -k 10 400 python -u scripts/ab_ragged.py rusty_enet_amd/lib/libenet_crc_amd.so \
  rusty_enet_amd/lib/variants/libenet_crc_amd_$V.so --configs $CFG --blocks $BLK > $O/ab_$V.txt 2> $O/ab_$V.err || { tail -20 $O/ab_$V.err; cat $O/ab_$V.txt; exit 1; }
grep -v "^{" $O/ab_$V.txt
echo "[variant] done"
