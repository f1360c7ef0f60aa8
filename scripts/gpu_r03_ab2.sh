#!/usr/bin/env bash
# Round-3 A/B 2: full GPU suite; G2/frag for the jobs kernel (ring 3, 8 slots; ring 4,
# 4 slots) and the region path (ring 3 / 4); counters of the jobs kernel and region4.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
P=rusty_enet_amd/lib/libenet_crc_amd.so
V=rusty_enet_amd/lib/variants
bash scripts/gpu_ab_configs.sh r03_ab2 "" "ragged frag" 2 $P $V/libenet_crc_amd_jobs4.so $V/libenet_crc_amd_region.so \
  $V/libenet_crc_amd_region4.so || exit $?
bash scripts/gpu_ragged_counters.sh r03_ab2/cnt_jobs $P || exit $?
bash scripts/gpu_ragged_counters.sh r03_ab2/cnt_region4 $V/libenet_crc_amd_region4.so || exit $?
