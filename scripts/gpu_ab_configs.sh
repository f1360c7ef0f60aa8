#!/usr/bin/env bash
# GPU parity tests (optional -k filter), then an alternating A/B of library builds
# (ENET_CRC_AMD_LIB) on bench configs, all in one gpurun call:
#   bash scripts/gpu_ab_configs.sh <tag> "<pytest -k expr or empty>" "<configs>" <reps> <libA.so> [<libB.so> ...]
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="$1"; K="$2"; CFGS="$3"; REPS="$4"; shift 4
OUT="$ROOT/gpurun_out/$TAG"
mkdir -p "$OUT"
cd "$ROOT"
if [ "$K" != "none" ]; then
  if [ -n "$K" ]; then
    timeout -k 10 600 python -u -m pytest tests -m gpu -q -k "$K" --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1
  else
    timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1
  fi
  rc=$?
  grep -E "^(FAILED|ERROR)" "$OUT/pytest.log" | head -20
  tail -2 "$OUT/pytest.log"
  # 1 = some tests failed: still time the builds; anything else (crash, timeout): stop
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
fi
for i in $(seq 1 "$REPS"); do
  for c in $CFGS; do
    for lib in "$@"; do
      name=$(basename "$lib" .so)
      ENET_CRC_AMD_LIB="$ROOT/$lib" timeout -k 10 150 python bench.py --config "$c" --cpu-seconds 0 --no-e2e \
        --no-shard --steps 60 > "$OUT/${c}_${name}_$i.json" 2> "$OUT/${c}_${name}_$i.err" || exit $?
      python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['roofline']['kernel_ms'], d['ms_per_step'], d['roofline']['frac'])" \
        "$OUT/${c}_${name}_$i.json" "$c $name run $i"
    done
  done
done
