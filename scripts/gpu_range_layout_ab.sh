#!/usr/bin/env bash
# Range-coder arena layout (ENET_RANGE_BLOCK = symbols per interleaved block; unset =
# one contiguous arena per coder): parity tests per layout, then alternating bench runs.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
OUT=gpurun_out/rlayout
mkdir -p $OUT
for v in 1 8; do
  ENET_RANGE_BLOCK=$v timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
    tests/test_gpu_range.py > $OUT/pytest_$v.log 2>&1 || { tail -30 $OUT/pytest_$v.log; exit 1; }
  tail -1 $OUT/pytest_$v.log
done
for i in 1 2; do
  for v in default 1 8; do
    if [ "$v" = default ]; then unset ENET_RANGE_BLOCK; else export ENET_RANGE_BLOCK=$v; fi
    timeout -k 10 200 python bench.py --config range --cpu-seconds 0 --steps 3 --warmup 1 \
      > $OUT/bench_${v}_$i.json 2> $OUT/bench_${v}_$i.err || exit $?
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['roofline'].get('kernel_ms'), d.get('decompress'))" \
      $OUT/bench_${v}_$i.json "BLOCK=$v run $i"
  done
done
