#!/bin/bash
# Round 5 working call: the GPU suite, the default bench line (now with verify_256), and the
# clock series of the clock-stamp build (with the same-box read ceiling).
#   gpurun --timeout 1200 -- bash scripts/gpu_r05_check.sh <tag> [pytest -k expression]
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
T=${1:-r05_check}
K=${2:-}
O=gpurun_out/$T
mkdir -p $O
if [ -n "$K" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread -k "$K" > $O/pytest_gpu.log 2>&1 || { tail -60 $O/pytest_gpu.log; exit 1; }
else
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -60 $O/pytest_gpu.log; exit 1; }
fi
tail -3 $O/pytest_gpu.log
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
python scripts/line_summary.py $O/bench.json
ENET_CRC_AMD_LIB=$PWD/rusty_enet_amd/lib/variants/libenet_crc_amd_clock.so CLOCK_SERIES_JSON=$O/clock_series.json \
  timeout -k 10 300 python -u scripts/exp_clock_series.py > $O/clock_series.txt 2> $O/clock_series.err || { tail -30 $O/clock_series.err; exit 1; }
echo "[check] done"
