#!/bin/bash
# The product build through the ragged GPU parity tests, then same-process A/Bs of variants
# (A) against the product (B).   gpurun -- bash scripts/gpu_r05_product_ab.sh <tag> <v1[,v2...]> [configs] [blocks]
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/$1
VS=$2
CFG=${3:-g2,frag,r740}
BLK=${4:-8}
K="ragged or frag or every_length or golden or host or ring or slot or full_size"
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_slot.py tests/test_gpu_ring.py -m gpu -x -q --timeout 240 --timeout-method thread -k "$K" > $O/pytest_product.log 2>&1 || { tail -40 $O/pytest_product.log; exit 1; }
tail -2 $O/pytest_product.log
for V in ${VS//,/ }; do
  timeout -k 10 400 python -u scripts/ab_ragged.py rusty_enet_amd/lib/variants/libenet_crc_amd_$V.so \
    rusty_enet_amd/lib/libenet_crc_amd.so --configs $CFG --blocks $BLK > $O/ab_${V}_vs_product.txt 2> $O/ab_$V.err || { tail -20 $O/ab_$V.err; cat $O/ab_${V}_vs_product.txt; exit 1; }
  echo "== $V (A) vs product (B)"; grep -v "^{" $O/ab_${V}_vs_product.txt
done
echo "[product_ab] done"
