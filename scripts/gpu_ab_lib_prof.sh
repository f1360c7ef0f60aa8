#!/usr/bin/env bash
# Kernel stats (rocprofv3 --kernel-trace --stats) of two library builds on one case of
# scripts/exp_ragged_overhead.py:  bash scripts/gpu_ab_lib_prof.sh <tag> <libA> <libB> <case>
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="$1"; A="$2"; B="$3"; CASE="$4"
OUT="$ROOT/gpurun_out/$TAG"
mkdir -p "$OUT"
export TMPDIR=/tmp
for i in 1 2; do
  for lib in "$A" "$B"; do
    name=$(basename "$lib" .so)
    ENET_CRC_AMD_LIB="$ROOT/$lib" timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$OUT/${name}_$i" -o run \
      --output-format csv -- python3 "$ROOT/scripts/exp_ragged_overhead.py" --reps 40 --only "$CASE" \
      > "$OUT/${name}_$i.log" 2>&1 || exit $?
    echo "== $name run $i"; grep -v amdgpu.ids "$OUT/${name}_$i.log" | grep " us "
    f=$(find "$OUT/${name}_$i" -name '*kernel_stats.csv' | head -1)
    python3 -c "
import csv,sys
for r in csv.DictReader(open(sys.argv[1])):
    print('   %-60s %8s calls  avg %.1f us' % (r['Name'][:60], r['Calls'], float(r['AverageNs'])/1e3))
" "$f"
  done
done
