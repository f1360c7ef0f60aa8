#!/usr/bin/env bash
# Ragged jobs kernel time split (stamps build) and the server latency experiment.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="${1:-r03_s3}"
OUT="$ROOT/gpurun_out/$TAG"
mkdir -p "$OUT"
cd "$ROOT"
ENET_CRC_AMD_LIB="$ROOT/rusty_enet_amd/lib/variants/libenet_crc_amd_stamps.so" timeout -k 10 170 \
  python scripts/exp_round_stamps.py > "$OUT/round_stamps.txt" 2>&1 || { tail -20 "$OUT/round_stamps.txt"; exit 1; }
grep -v amdgpu.ids "$OUT/round_stamps.txt"
timeout -k 10 120 python scripts/exp_server_latency.py > "$OUT/server_latency.txt" 2>&1 || { tail -20 "$OUT/server_latency.txt"; exit 1; }
grep -v amdgpu.ids "$OUT/server_latency.txt"
