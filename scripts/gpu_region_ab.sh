#!/usr/bin/env bash
# Smaller sort regions for the ragged pre-pass (ENET_CRC_REGION): parity, then A/B on G2.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
OUT=gpurun_out/region
mkdir -p $OUT
ENET_CRC_REGION=1024 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py -k "ragged" > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for i in 1 2 3; do
  for v in default 2048 1024; do
    if [ "$v" = default ]; then unset ENET_CRC_REGION; else export ENET_CRC_REGION=$v; fi
    timeout -k 10 200 python bench.py --config ragged --cpu-seconds 0 --no-e2e --steps 100 \
      > $OUT/bench_${v}_$i.json 2> $OUT/bench_${v}_$i.err || exit $?
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['roofline']['kernel_ms'], d['ms_per_step'], d['roofline']['frac'])" \
      $OUT/bench_${v}_$i.json "REGION=$v run $i"
  done
done
