#!/bin/bash
# The clock series on the product build and on the (atomic-free) clock-stamp build.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-r05_clock3}
mkdir -p $O
ENET_CRC_AMD_LIB=$PWD/rusty_enet_amd/lib/variants/libenet_crc_amd_clock.so CLOCK_SERIES_JSON=$O/clock.json \
  timeout -k 10 300 python -u scripts/exp_clock_series.py > $O/clock.txt 2> $O/clock.err || { tail -30 $O/clock.err; exit 1; }
CLOCK_SERIES_JSON=$O/product.json timeout -k 10 300 python -u scripts/exp_clock_series.py > $O/product.txt 2> $O/product.err || { tail -30 $O/product.err; exit 1; }
echo "[clock3] done"
