#!/usr/bin/env bash
# Persistent server next to batches: hooks and multi GPU tests, then the latency experiment.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="${1:-r03_s4}"
OUT="$ROOT/gpurun_out/$TAG"
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_hooks.py tests/test_gpu_multi.py -m gpu -q -x --timeout 200 \
  --timeout-method thread > "$OUT/pytest_server.log" 2>&1 || { tail -30 "$OUT/pytest_server.log"; exit 1; }
tail -1 "$OUT/pytest_server.log"
timeout -k 10 120 python scripts/exp_server_latency.py > "$OUT/server_latency.txt" 2>&1 || { tail -20 "$OUT/server_latency.txt"; exit 1; }
grep -v amdgpu.ids "$OUT/server_latency.txt"
