#!/bin/bash
# Same-process A/Bs of variant builds (A) against the product (B) on the ragged configs, each
# variant's output checked against the product's in full and against the oracle on a sample
# (scripts/ab_ragged.py).   gpurun -- bash scripts/gpu_r06_ab.sh <tag> <v1[,v2...]> [configs] [blocks]
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/$1
VS=$2
CFG=${3:-g2,frag,r740}
BLK=${4:-12}
mkdir -p $O
for V in ${VS//,/ }; do
  timeout -k 10 400 python -u scripts/ab_ragged.py rusty_enet_amd/lib/variants/libenet_crc_amd_$V.so \
    rusty_enet_amd/lib/libenet_crc_amd.so --configs $CFG --blocks $BLK > $O/ab_${V}_vs_product.txt 2> $O/ab_$V.err || { tail -20 $O/ab_$V.err; cat $O/ab_${V}_vs_product.txt; exit 1; }
  echo "== $V (A) vs product (B)"; grep -v "^{" $O/ab_${V}_vs_product.txt
done
echo "[r06_ab] done"
