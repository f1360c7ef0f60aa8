#!/bin/bash
# Same-process A/B of the product against a variant build (scripts/ab_ragged.py), plus
# optional extra commands.   gpurun -- bash scripts/gpu_r05_ab.sh <tag> <variant name> [configs] [blocks]
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/$1
V=$2
CFG=${3:-g2,frag,r740}
BLK=${4:-8}
mkdir -p $O
timeout -k 10 400 python -u scripts/ab_ragged.py rusty_enet_amd/lib/libenet_crc_amd.so \
  rusty_enet_amd/lib/variants/libenet_crc_amd_$V.so --configs $CFG --blocks $BLK > $O/ab_$V.txt 2> $O/ab_$V.err || { tail -20 $O/ab_$V.err; cat $O/ab_$V.txt; exit 1; }
grep -v "^{" $O/ab_$V.txt
if [ -n "${STAMPS:-}" ]; then
  ENET_CRC_AMD_LIB=$PWD/rusty_enet_amd/lib/variants/libenet_crc_amd_stamps.so timeout -k 10 300 python -u scripts/exp_round_stamps.py > $O/round_stamps.txt 2>&1 || { tail -20 $O/round_stamps.txt; exit 1; }
  cat $O/round_stamps.txt
fi
echo "[ab] done"
