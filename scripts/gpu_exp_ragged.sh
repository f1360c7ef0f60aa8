#!/usr/bin/env bash
# Ragged main-kernel time under ENET_CRC_EXP values (timing experiments): bash scripts/gpu_exp_ragged.sh <tag> <v1> <v2> ...
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/$1"; shift
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
i=0
for v in "$@"; do
  i=$((i+1))
  export ENET_CRC_EXP=$v
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_$i" -o run --output-format csv \
    -- python3 "$ROOT/bench.py" --config ragged --steps 20 --warmup 2 --cpu-seconds 0 --no-verify --no-e2e --no-shard \
    > "$OUT/prof_$i.log" 2>&1 || exit $?
  python3 - "$OUT/prof_$i/run_kernel_stats.csv" "$v" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if 'ragged_dma' in r['Name']: print("exp", sys.argv[2], r['AverageNs'], r['MinNs'], r['MaxNs'])
PY
done
