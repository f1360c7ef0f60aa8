#!/usr/bin/env bash
# Quick GPU iteration: parity tests (all, or those matching $2), then the bench line of
# each config listed in $3 (default "ragged").  Usage: gpu_quick.sh <tag> [pytest -k expr] [configs]
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="${1:-quick}"; K="${2:-}"; CFGS="${3:-ragged}"
OUT="$ROOT/gpurun_out/$TAG"
mkdir -p "$OUT"
cd "$ROOT"
if [ -n "$K" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -k "$K" --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1
else
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1
fi
rc=$?
tail -3 "$OUT/pytest.log"
[ $rc -eq 0 ] || exit $rc
for c in $CFGS; do
  timeout -k 10 200 python bench.py --config $c --cpu-seconds 0 --no-e2e --no-shard > "$OUT/bench_$c.json" 2> "$OUT/bench_$c.err" || exit $?
  python3 -c "import json; d=json.load(open('$OUT/bench_$c.json')); print('$c', d['value'], d['roofline']['kernel_ms'], d['roofline']['frac'])"
done
