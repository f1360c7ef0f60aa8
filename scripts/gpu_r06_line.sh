#!/bin/bash
# Round 6 line rounds: the product (line rounds on) through the ragged GPU parity tests, then a
# same-process A/B against the same source with line rounds off (variants/..._line0.so).
#   gpurun -- bash scripts/gpu_r06_line.sh <tag> [configs] [blocks]
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/$1
CFG=${2:-frag,g2,r1392,r740}
BLK=${3:-12}
K="ragged or frag or every_length or golden or host or ring or slot or full_size"
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_slot.py tests/test_gpu_ring.py -m gpu -x -q --timeout 240 --timeout-method thread -k "$K" > $O/pytest_product.log 2>&1 || { tail -40 $O/pytest_product.log; exit 1; }
tail -2 $O/pytest_product.log
timeout -k 10 500 python -u scripts/ab_ragged.py rusty_enet_amd/lib/libenet_crc_amd.so \
  rusty_enet_amd/lib/variants/libenet_crc_amd_line0.so --configs $CFG --blocks $BLK > $O/ab_line_vs_line0.txt 2> $O/ab.err || { tail -20 $O/ab.err; cat $O/ab_line_vs_line0.txt; exit 1; }
echo "== product, line rounds (A) vs line rounds off (B)"; grep -v "^{" $O/ab_line_vs_line0.txt
echo "[line] done"
