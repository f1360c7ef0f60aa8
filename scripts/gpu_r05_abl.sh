#!/bin/bash
# Ablation A/Bs (B builds compute wrong checksums: --unchecked-b): product vs each named variant.
#   gpurun -- bash scripts/gpu_r05_abl.sh <tag> <configs> <variant>...
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/$1; CFG=$2; shift 2
mkdir -p $O
for V in "$@"; do
  timeout -k 10 300 python -u scripts/ab_ragged.py rusty_enet_amd/lib/libenet_crc_amd.so \
    rusty_enet_amd/lib/variants/libenet_crc_amd_$V.so --configs $CFG --blocks 8 --unchecked-b > $O/ab_$V.txt 2> $O/ab_$V.err || { tail -20 $O/ab_$V.err; exit 1; }
  echo "== $V"; grep -v "^{" $O/ab_$V.txt
done
