#!/usr/bin/env bash
# Line-split LDS-DMA ring with shared lines read once (ENET_CRC_UNIFORM=dmas): parity,
# then alternating G1 runs against the default register ring.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
OUT=gpurun_out/dmas
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py -k "shared_lines_dma or dmas" > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for i in 1 2 3 4; do
  for v in default dmas; do
    if [ "$v" = default ]; then unset ENET_CRC_UNIFORM; else export ENET_CRC_UNIFORM=$v; fi
    timeout -k 10 200 python bench.py --config uniform --cpu-seconds 0 --no-e2e --no-shard --steps 40 \
      > $OUT/bench_${v}_$i.json 2> $OUT/bench_${v}_$i.err || exit $?
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['roofline']['kernel_ms'], d['ms_per_step'], d['roofline']['frac'])" \
      $OUT/bench_${v}_$i.json "UNIFORM=$v run $i"
  done
done
