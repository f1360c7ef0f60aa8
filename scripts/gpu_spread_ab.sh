#!/usr/bin/env bash
# Spread packet mapping (ENET_CRC_SPREAD=1) in the register kernel: uniform parity tests
# with the switch on, then alternating A/B on G1.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
mkdir -p gpurun_out/spread
ENET_CRC_SPREAD=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py -k "uniform or shard_uniform or line_split" > gpurun_out/spread/pytest.log 2>&1 || { tail -30 gpurun_out/spread/pytest.log; exit 1; }
tail -2 gpurun_out/spread/pytest.log
bash scripts/gpu_ab_env.sh spread uniform ENET_CRC_SPREAD default 1 4
