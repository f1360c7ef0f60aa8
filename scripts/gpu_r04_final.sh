#!/bin/bash
# Round 4 evidence, part 1: the GPU suite, the driver's bench command and the default bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-r04_final}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -60 $O/pytest_gpu.log; exit 1; }
tail -3 $O/pytest_gpu.log
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_20_5.json 2> $O/bench_20_5.err || exit $?
python scripts/line_summary.py $O/bench_20_5.json
timeout -k 10 300 python -u bench.py > $O/bench_default.json 2> $O/bench_default.err || exit $?
python scripts/line_summary.py $O/bench_default.json
bash scripts/gpu_r04_pair.sh ${1:-r04_final} || exit $?
