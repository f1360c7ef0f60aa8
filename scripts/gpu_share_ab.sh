#!/usr/bin/env bash
# Shared boundary lines (ENET_CRC_SHARE=1|2|3) in the line-split register kernel: parity
# tests with the switch, then alternating runs on G1 against the default.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
OUT=gpurun_out/share
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py -k "shared_boundary or uniform_batch or full_size_uniform or shard_uniform" > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
for i in 1 2 3; do
  for v in default 1 2 3; do
    if [ "$v" = default ]; then unset ENET_CRC_SHARE; else export ENET_CRC_SHARE=$v; fi
    timeout -k 10 200 python bench.py --config uniform --cpu-seconds 0 --no-e2e --no-shard --steps 40 \
      > $OUT/bench_${v}_$i.json 2> $OUT/bench_${v}_$i.err || exit $?
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['roofline']['kernel_ms'], d['ms_per_step'])" \
      $OUT/bench_${v}_$i.json "SHARE=$v run $i"
  done
done
