#!/usr/bin/env bash
# Wave-per-packet kernel for long packets (ENET_CRC_LONG=wave): parity tests, then
# alternating runs on the 64-KiB config (G4 shard) against the default.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
OUT=gpurun_out/wave
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py -k "wave or large or long_packets" > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
for i in 1 2 3; do
  for v in default wave; do
    if [ "$v" = default ]; then unset ENET_CRC_LONG; else export ENET_CRC_LONG=$v; fi
    timeout -k 10 200 python bench.py --config large --cpu-seconds 0 --no-e2e --steps 40 \
      > $OUT/bench_${v}_$i.json 2> $OUT/bench_${v}_$i.err || exit $?
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['roofline']['kernel_ms'], d['ms_per_step'], d['roofline']['frac'])" \
      $OUT/bench_${v}_$i.json "LONG=$v run $i"
  done
done
