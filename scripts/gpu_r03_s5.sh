#!/usr/bin/env bash
# Device-side kick: full GPU suite, the server latency experiment, and the uniform/ragged
# bench configs (the kick costs one load and store per launch).
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="${1:-r03_s5}"
OUT="$ROOT/gpurun_out/$TAG"
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
  > "$OUT/pytest_gpu.log" 2>&1 || { tail -30 "$OUT/pytest_gpu.log"; exit 1; }
tail -1 "$OUT/pytest_gpu.log"
timeout -k 10 120 python scripts/exp_server_latency.py > "$OUT/server_latency.txt" 2>&1 || { tail -20 "$OUT/server_latency.txt"; exit 1; }
grep -v amdgpu.ids "$OUT/server_latency.txt"
for c in uniform ragged; do
  timeout -k 10 200 python bench.py --config $c --cpu-seconds 0 --no-e2e --no-shard --steps 100 > "$OUT/bench_$c.json" 2> "$OUT/bench_$c.err" || exit $?
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['roofline']['kernel_ms'], d['ms_per_step'], d['roofline']['frac'])" "$OUT/bench_$c.json" $c
done
ENET_CRC_AMD_LIB="$ROOT/rusty_enet_amd/lib/variants/libenet_crc_amd_stamps.so" timeout -k 10 170 \
  python scripts/exp_round_stamps.py > "$OUT/round_stamps.txt" 2>&1 || { tail -20 "$OUT/round_stamps.txt"; exit 1; }
grep -v amdgpu.ids "$OUT/round_stamps.txt"
