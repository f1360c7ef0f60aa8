#!/usr/bin/env bash
# A/B of the XCD-aware round order on the 64-KiB config, alternating in one call.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/${1:-abxcdl}"
mkdir -p "$OUT"
cd "$ROOT"
for i in 1 2 3; do
  for x in 0 1; do
    ENET_CRC_XCD=$x timeout -k 10 200 python bench.py --config large --cpu-seconds 0 --no-e2e --steps 40 > "$OUT/bench_x${x}_$i.json" 2>/dev/null || exit $?
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['roofline']['kernel_ms'])" "$OUT/bench_x${x}_$i.json" "large x=$x run $i"
    ENET_CRC_XCD=$x timeout -k 10 200 python bench.py --cpu-seconds 0 --no-e2e --no-shard --steps 40 > "$OUT/ubench_x${x}_$i.json" 2>/dev/null || exit $?
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['roofline']['kernel_ms'])" "$OUT/ubench_x${x}_$i.json" "uniform x=$x run $i"
  done
done
