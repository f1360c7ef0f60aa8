#!/bin/bash
# Instruction-cache counters of the product kernels (G1 whole-line, G2 ragged, frag_64k):
# one rocprofv3 --pmc pass of 8 SQ-block counters per config.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/${1:-r05_icache}"
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
for c in uniform ragged frag; do
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES \
    SQC_ICACHE_MISSES_DUPLICATE SQC_ICACHE_INPUT_VALID_READYB SQ_IFETCH SQ_WAIT_INST_ANY SQ_BUSY_CYCLES \
    -d "$OUT/ic_$c" -o run --output-format csv \
    -- python3 "$ROOT/bench.py" --config $c --steps 5 --warmup 1 --cpu-seconds 0 --no-verify --no-e2e --no-shard \
    > "$OUT/ic_$c.log" 2>&1 || exit $?
  echo "[icache] $c done" >&2
done
cd "$ROOT"
for c in uniform ragged frag; do
  python3 scripts/pmc_summary.py "$OUT/ic_$c" > "$OUT/ic_${c}_summary.txt" 2>&1
done
echo "[icache] done" >&2
