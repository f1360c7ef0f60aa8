#!/usr/bin/env bash
# Round-3 A/B 4: full GPU suite; uniform parity on the shared-line DMA variant; G1 with the
# replicated tree block vs unreplicated vs the shared-line DMA variants; G2/frag vs the
# region path; the server-overlap experiment; uniform and ragged counters.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
P=rusty_enet_amd/lib/libenet_crc_amd.so
V=rusty_enet_amd/lib/variants
mkdir -p gpurun_out/r03_ab4
bash scripts/gpu_ab_configs.sh r03_ab4 "" "uniform" 3 $P $V/libenet_crc_amd_unrep.so $V/libenet_crc_amd_lines1.so \
  $V/libenet_crc_amd_lines2.so || exit $?
ENET_CRC_AMD_LIB="$ROOT/$V/libenet_crc_amd_lines1.so" timeout -k 10 170 python -u -m pytest tests -m gpu -q \
  -k "uniform or line_split or 1200 or shapes or full_shard or bit_flip or long" --timeout 150 --timeout-method thread \
  > gpurun_out/r03_ab4/pytest_lines1.log 2>&1; echo "lines1 pytest rc=$?"; tail -2 gpurun_out/r03_ab4/pytest_lines1.log
bash scripts/gpu_ab_configs.sh r03_ab4r none "ragged frag" 2 $P $V/libenet_crc_amd_region.so || exit $?
ENET_CRC_AMD_LIB="$ROOT/$V/libenet_crc_amd_testhooks.so" timeout -k 10 150 python scripts/exp_server_overlap.py \
  > gpurun_out/r03_ab4/server_overlap.txt 2>&1 || exit $?
cat gpurun_out/r03_ab4/server_overlap.txt
bash scripts/gpu_ragged_counters.sh r03_ab4/cnt_uniform $P uniform || exit $?
bash scripts/gpu_ragged_counters.sh r03_ab4/cnt_jobs $P ragged || exit $?
