#!/bin/bash
# The clock series on the product build and on the clock-stamp build, one process each, and a
# kernel trace of the stamp build's series (do the stamps themselves change the kernels?).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-r05_clock2}
mkdir -p $O
CLOCK_SERIES_JSON=$O/product.json timeout -k 10 300 python -u scripts/exp_clock_series.py > $O/product.txt 2> $O/product.err || { tail -30 $O/product.err; exit 1; }
ENET_CRC_AMD_LIB=$PWD/rusty_enet_amd/lib/variants/libenet_crc_amd_clock.so CLOCK_SERIES_JSON=$O/clock.json \
  timeout -k 10 300 python -u scripts/exp_clock_series.py > $O/clock.txt 2> $O/clock.err || { tail -30 $O/clock.err; exit 1; }
export TMPDIR=/tmp
(cd /tmp && ENET_CRC_AMD_LIB=$GRAFT_REPO_ROOT/rusty_enet_amd/lib/variants/libenet_crc_amd_clock.so timeout -k 10 300 \
  rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/trace_clock -o run --output-format csv \
  -- python3 $GRAFT_REPO_ROOT/scripts/exp_clock_series.py > $GRAFT_REPO_ROOT/$O/trace_clock.log 2>&1) || exit 1
echo "[clock2] done"
