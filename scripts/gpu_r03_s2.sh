#!/usr/bin/env bash
# Round-3 diagnostics in one call: job-flag polling of the ragged jobs kernel (spin
# build), ragged-vs-uniform per-round overhead, and the G1 counter diff against probe P9.
#   gpurun --timeout 900 -- bash scripts/gpu_r03_s2.sh <tag>
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="${1:-r03_s2}"
OUT="$ROOT/gpurun_out/$TAG"
mkdir -p "$OUT"
cd "$ROOT"
ENET_CRC_AMD_LIB="$ROOT/rusty_enet_amd/lib/variants/libenet_crc_amd_spin.so" timeout -k 10 170 \
  python scripts/exp_spin_stats.py > "$OUT/spin_stats.txt" 2>&1 || { tail -20 "$OUT/spin_stats.txt"; exit 1; }
cat "$OUT/spin_stats.txt"
timeout -k 10 200 python scripts/exp_ragged_overhead.py --reps 30 > "$OUT/ragged_overhead.txt" 2>&1 \
  || { tail -20 "$OUT/ragged_overhead.txt"; exit 1; }
cat "$OUT/ragged_overhead.txt"
bash scripts/gpu_g1_diff.sh "$TAG/g1diff"
ENET_CRC_AMD_LIB="$ROOT/rusty_enet_amd/lib/variants/libenet_crc_amd_testhooks.so" timeout -k 10 170 \
  python scripts/exp_server_overlap.py > "$OUT/server_overlap.txt" 2>&1 || { tail -20 "$OUT/server_overlap.txt"; exit 1; }
cat "$OUT/server_overlap.txt"
