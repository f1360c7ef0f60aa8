#!/usr/bin/env bash
# Round-3 A/B 5: the server-overlap experiment with stream-only syncs, the hooks tests,
# and G2/frag with the makespan-minimising job size.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
P=rusty_enet_amd/lib/libenet_crc_amd.so
V=rusty_enet_amd/lib/variants
mkdir -p gpurun_out/r03_ab5
ENET_CRC_AMD_LIB="$ROOT/$V/libenet_crc_amd_testhooks.so" timeout -k 10 150 python scripts/exp_server_overlap.py \
  > gpurun_out/r03_ab5/server_overlap.txt 2>&1 || exit $?
cat gpurun_out/r03_ab5/server_overlap.txt
bash scripts/gpu_ab_configs.sh r03_ab5 "hooks or ragged or slot or multi" "ragged frag" 2 $P $V/libenet_crc_amd_region.so
