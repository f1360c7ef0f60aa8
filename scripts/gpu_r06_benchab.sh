#!/bin/bash
# bench.py --config <c> alternating between the product and a variant build (ENET_CRC_AMD_LIB),
# so sustained and cold numbers come from the bench's own harness.  Optional parity subset first.
#   gpurun -- bash scripts/gpu_r06_benchab.sh <tag> <variant> [configs] [rounds]
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/$1
V=$2
CFGS=${3:-frag,ragged}
N=${4:-2}
mkdir -p $O
if [ "${PARITY:-0}" = 1 ]; then
  K="ragged or frag or every_length or golden or host or ring or slot or full_size"
  timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_slot.py tests/test_gpu_ring.py -m gpu -x -q --timeout 240 --timeout-method thread -k "$K" > $O/pytest_product.log 2>&1 || { tail -40 $O/pytest_product.log; exit 1; }
  tail -1 $O/pytest_product.log
fi
for c in ${CFGS//,/ }; do
  for i in $(seq 1 $N); do
    for w in product $V; do
      if [ $w = product ]; then unset ENET_CRC_AMD_LIB; else export ENET_CRC_AMD_LIB=$PWD/rusty_enet_amd/lib/variants/libenet_crc_amd_$w.so; fi
      timeout -k 10 200 python -u bench.py --config $c --steps 200 --warmup 10 --cpu-seconds 0 --no-e2e > $O/bench_${c}_${w}_$i.json 2> $O/bench_${c}_${w}_$i.err || { tail -5 $O/bench_${c}_${w}_$i.err; exit 1; }
    done
  done
done
unset ENET_CRC_AMD_LIB
python scripts/line_summary.py $O/bench_*.json
echo "[benchab] done"
