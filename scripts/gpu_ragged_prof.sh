#!/usr/bin/env bash
# Kernel stats and FETCH_SIZE of the ragged config for ENET_CRC_RAGGED=global and the default.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/${1:-ragprof}"
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
for m in global default; do
  if [ $m = default ]; then unset ENET_CRC_RAGGED; else export ENET_CRC_RAGGED=$m; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_$m" -o run --output-format csv \
    -- python3 "$ROOT/bench.py" --config ragged --steps 20 --warmup 2 --cpu-seconds 0 --no-verify --no-e2e --no-shard \
    > "$OUT/prof_$m.log" 2>&1 || exit $?
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d "$OUT/pmc_$m" -o run --output-format csv \
    -- python3 "$ROOT/bench.py" --config ragged --steps 5 --warmup 1 --cpu-seconds 0 --no-verify --no-e2e --no-shard \
    > "$OUT/pmc_$m.log" 2>&1 || exit $?
  echo "[ragprof] $m done" >&2
done
unset ENET_CRC_RAGGED
cd "$ROOT"
for m in global default; do
  echo "== $m"
  f=$(ls "$OUT"/prof_$m/run_kernel_stats.csv "$OUT"/prof_$m/*/run_kernel_stats.csv 2>/dev/null | head -1)
  [ -n "$f" ] && cut -d, -f1-4 "$f" | grep -i crc | cut -c1-160
  python3 scripts/pmc_summary.py "$OUT"/pmc_$m 2>/dev/null | grep -A1 -i "crc" | head -12
done
