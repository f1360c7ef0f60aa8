#!/usr/bin/env bash
# Round-3 A/B 3: full GPU suite; G2/frag jobs kernel (no spills) vs the region path;
# jobs-kernel counters; then the G1 ceiling counters (probe P9 vs the G1 kernel).
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
P=rusty_enet_amd/lib/libenet_crc_amd.so
V=rusty_enet_amd/lib/variants
bash scripts/gpu_ab_configs.sh r03_ab3 "" "ragged frag" 2 $P $V/libenet_crc_amd_region.so || exit $?
bash scripts/gpu_ragged_counters.sh r03_ab3/cnt_jobs $P || exit $?
bash scripts/gpu_g1_diff.sh r03_g1diff || exit $?
