#!/bin/bash
# Round 4: the new mixed-class ragged round parity tests on the product, then the whole suite.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-r04_mixed}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -60 $O/pytest_gpu.log; exit 1; }
grep -E "mixed_class|passed|failed" $O/pytest_gpu.log | tail -6
