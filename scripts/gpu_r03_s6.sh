#!/usr/bin/env bash
# Ragged per-round overhead cut (4-trip combine, one-trip record read, no-wait result store,
# 6 job slots) and the device-side server kick: full GPU suite, server latency experiment,
# round stamps, then ragged/frag A/B against the previous commit's build (prev).
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="${1:-r03_s6}"
OUT="$ROOT/gpurun_out/$TAG"
mkdir -p "$OUT"
cd "$ROOT"
V=rusty_enet_amd/lib/variants
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
  > "$OUT/pytest_gpu.log" 2>&1 || { tail -30 "$OUT/pytest_gpu.log"; exit 1; }
tail -1 "$OUT/pytest_gpu.log"
timeout -k 10 120 python scripts/exp_server_latency.py > "$OUT/server_latency.txt" 2>&1 || { tail -20 "$OUT/server_latency.txt"; exit 1; }
grep -v amdgpu.ids "$OUT/server_latency.txt"
ENET_CRC_AMD_LIB="$ROOT/$V/libenet_crc_amd_stamps.so" timeout -k 10 170 \
  python scripts/exp_round_stamps.py > "$OUT/round_stamps.txt" 2>&1 || { tail -20 "$OUT/round_stamps.txt"; exit 1; }
grep -v amdgpu.ids "$OUT/round_stamps.txt"
bash scripts/gpu_ab_configs.sh "$TAG" none "ragged frag" 3 rusty_enet_amd/lib/libenet_crc_amd.so $V/libenet_crc_amd_prev.so
