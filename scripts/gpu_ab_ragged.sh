#!/usr/bin/env bash
# A/B of the ragged paths (ENET_CRC_RAGGED modes) with kernel stats per mode.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="${1:-abr}"; shift || true
MODES="${*:-segment global}"
OUT="$ROOT/gpurun_out/$TAG"
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -k "ragged or alternative or every_length or golden" --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { tail -20 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
export TMPDIR=/tmp
for m in $MODES; do
  ( cd /tmp && ENET_CRC_RAGGED=$m timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$OUT/prof_$m" -o run --output-format csv \
    -- python3 "$ROOT/bench.py" --config ragged --steps 20 --warmup 3 --cpu-seconds 0 --no-verify --no-e2e > "$OUT/prof_$m.log" 2>&1 ) || exit $?
  python3 - "$OUT/prof_$m" "$m" <<'PY'
import csv, glob, sys
for f in glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "crc32" in r["Name"]:
            print(sys.argv[2], r["Name"].split("(")[0].split("::")[-1][:40], r["Calls"], round(float(r["AverageNs"]) / 1e3, 1), "us")
PY
done
