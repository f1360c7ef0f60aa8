#!/usr/bin/env bash
# Round-3 A/B 4: full GPU suite; G1 with the replicated tree block vs unreplicated; G2/frag
# (job flags polled once per job) vs the region path; uniform counters (bank conflicts).
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
P=rusty_enet_amd/lib/libenet_crc_amd.so
V=rusty_enet_amd/lib/variants
bash scripts/gpu_ab_configs.sh r03_ab4 "" "uniform" 3 $P $V/libenet_crc_amd_unrep.so || exit $?
bash scripts/gpu_ab_configs.sh r03_ab4r none "ragged frag" 2 $P $V/libenet_crc_amd_region.so || exit $?
bash scripts/gpu_ragged_counters.sh r03_ab4/cnt_uniform $P uniform || exit $?
bash scripts/gpu_ragged_counters.sh r03_ab4/cnt_jobs $P ragged || exit $?
mkdir -p gpurun_out/r03_ab4
ENET_CRC_AMD_LIB="$ROOT/$V/libenet_crc_amd_testhooks.so" timeout -k 10 150 python scripts/exp_server_overlap.py \
  > gpurun_out/r03_ab4/server_overlap.txt 2>&1 || exit $?
cat gpurun_out/r03_ab4/server_overlap.txt
