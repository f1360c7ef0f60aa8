#!/bin/bash
# The whole GPU suite and smoke() on the product, then same-process A/Bs of variants (A)
# against it (B).   gpurun -- bash scripts/gpu_r05_suite_ab.sh <tag> <v1[,v2...]> [configs] [blocks]
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/$1
VS=$2
CFG=${3:-g2,frag,r740}
BLK=${4:-12}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -60 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
for V in ${VS//,/ }; do
  timeout -k 10 400 python -u scripts/ab_ragged.py rusty_enet_amd/lib/variants/libenet_crc_amd_$V.so \
    rusty_enet_amd/lib/libenet_crc_amd.so --configs $CFG --blocks $BLK > $O/ab_${V}_vs_product.txt 2> $O/ab_$V.err || { tail -20 $O/ab_$V.err; cat $O/ab_${V}_vs_product.txt; exit 1; }
  echo "== $V (A) vs product (B)"; grep -v "^{" $O/ab_${V}_vs_product.txt
done
echo "[suite_ab] done"
