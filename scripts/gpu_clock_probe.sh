set -u
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for b in base no_mem no_compute; do
  timeout -k 5 120 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE -d $R/gpurun_out/clk_$b -o run --output-format csv -- $R/tools/ablate/bin/$b > /dev/null 2>&1 || exit 1
done
timeout -k 5 120 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE -d $R/gpurun_out/clk_probe -o run --output-format csv -- $R/tools/read_probe > /dev/null 2>&1 || exit 1
echo done
