#!/usr/bin/env bash
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
V=rusty_enet_amd/lib/variants
mkdir -p gpurun_out/r03_ab6
ENET_CRC_AMD_LIB="$ROOT/$V/libenet_crc_amd_testhooks.so" timeout -k 10 170 python scripts/exp_server_overlap.py \
  > gpurun_out/r03_ab6/server_overlap.txt 2>&1
rc=$?
cat gpurun_out/r03_ab6/server_overlap.txt
exit $rc
