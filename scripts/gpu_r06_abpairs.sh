#!/bin/bash
# Same-process A/Bs of library pairs (scripts/ab_ragged.py: outputs compared in full and
# against the oracle on a sample).  Pairs "A:B,..."; a name is a variant build
# (variants/libenet_crc_amd_<name>.so) or "product".  Optional parity subset first (PARITY=1).
#   gpurun -- bash scripts/gpu_r06_abpairs.sh <tag> <pairs> [configs] [blocks]
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/$1
PAIRS=$2
CFG=${3:-frag,g2,r1392,r740}
BLK=${4:-12}
mkdir -p $O
lib() { if [ "$1" = product ]; then echo rusty_enet_amd/lib/libenet_crc_amd.so; else echo rusty_enet_amd/lib/variants/libenet_crc_amd_$1.so; fi; }
if [ "${PARITY:-0}" = 1 ]; then
  K="ragged or frag or every_length or golden or host or ring or slot or full_size"
  timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_slot.py tests/test_gpu_ring.py -m gpu -x -q --timeout 240 --timeout-method thread -k "$K" > $O/pytest_product.log 2>&1 || { tail -40 $O/pytest_product.log; exit 1; }
  tail -1 $O/pytest_product.log
fi
for P in ${PAIRS//,/ }; do
  A=${P%%:*}; B=${P##*:}
  timeout -k 10 500 python -u scripts/ab_ragged.py $(lib $A) $(lib $B) --configs $CFG --blocks $BLK > $O/ab_${A}_vs_$B.txt 2> $O/ab_${A}_$B.err || { tail -20 $O/ab_${A}_$B.err; cat $O/ab_${A}_vs_$B.txt; exit 1; }
  echo "== $A (A) vs $B (B)"; grep -v "^{" $O/ab_${A}_vs_$B.txt | sed 's/ us  B \[.*\] us  -> / -> /; s/: A \[.*\] us  B/: /'
done
echo "[abpairs] done"
