#!/usr/bin/env bash
# Round-3 A/B: full GPU suite, then ragged/frag (jobs kernel vs region pre-pass) and
# uniform (register ring vs the time-aligned line DMA variants), alternating, one call.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
P=rusty_enet_amd/lib/libenet_crc_amd.so
V=rusty_enet_amd/lib/variants
bash scripts/gpu_ab_configs.sh r03_ab1 "" "ragged frag" 2 $P $V/libenet_crc_amd_region.so $V/libenet_crc_amd_nomixed.so || exit $?
bash scripts/gpu_ab_configs.sh r03_ab1u none "uniform" 2 $P $V/libenet_crc_amd_lines0.so $V/libenet_crc_amd_lines1.so $V/libenet_crc_amd_lines2.so
