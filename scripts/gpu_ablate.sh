#!/usr/bin/env bash
# Time every tools/ablate/bin/* variant (DMA and register-ring uniform kernels), then
# read each one's effective clock with rocprofv3 (GRBM_GUI_ACTIVE / duration).
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
for b in "$R"/tools/ablate/bin/*; do timeout -k 5 60 "$b" || exit 1; done
for b in "$R"/tools/ablate/bin/*; do ENET_CRC_UNIFORM=regs timeout -k 5 60 "$b" | sed 's/^/regs:/' || exit 1; done
cd /tmp && export TMPDIR=/tmp
for b in "$R"/tools/ablate/bin/*; do
  n=$(basename "$b")
  timeout -k 5 120 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE -d "$R/gpurun_out/clk_$n" -o run --output-format csv -- "$b" > /dev/null 2>&1 || exit 1
done
python3 "$R/scripts/clock_summary.py" "$R"/gpurun_out/clk_*
