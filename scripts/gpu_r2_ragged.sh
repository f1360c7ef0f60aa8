#!/usr/bin/env bash
# Round-2 check of the group-stream ragged kernel: GPU parity tests, then A/B bench of
# the ragged config (group-stream default vs the sorted round kernel) and the uniform line.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="${1:-r2gs}"
OUT="$ROOT/gpurun_out/$TAG"
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?
echo "pytest rc=$rc" >> "$OUT/pytest.log"
tail -3 "$OUT/pytest.log"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python bench.py --config ragged --cpu-seconds 0 --no-e2e > "$OUT/bench_ragged_gs.json" 2> "$OUT/bench_ragged_gs.err" || exit $?
ENET_CRC_RAGGED=sorted timeout -k 10 200 python bench.py --config ragged --cpu-seconds 0 --no-e2e > "$OUT/bench_ragged_sorted.json" 2> "$OUT/bench_ragged_sorted.err" || exit $?
for f in "$OUT"/bench_ragged_*.json; do python3 -c "import json,sys; d=json.load(open('$f')); print('$f', d['value'], d['roofline']['kernel_ms'], d['roofline']['frac'])"; done
