#!/usr/bin/env bash
# Run GPU steps one after another (each under its own time limit); stop at the first
# step that fails, faults (the HIP runtime prints HSA_STATUS_ERROR even when the process
# exits 0) or times out.  Output of step i goes to gpurun_out/steps/<i>.log.
#   gpurun -- bash scripts/gpu_steps.sh <seconds-per-step> 'cmd1' 'cmd2' ...
set -u
T="$1"; shift
R="${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p "$R/gpurun_out/steps"
i=0
for c in "$@"; do
  i=$((i + 1))
  log="$R/gpurun_out/steps/$i.log"
  timeout -k 10 "$T" bash -c "$c" > "$log" 2>&1
  rc=$?
  cat "$log"
  if [ $rc -ne 0 ] || grep -q "HSA_STATUS_ERROR\|hardware exception\|Memory access fault" "$log"; then
    echo "[gpu_steps] step $i failed (rc=$rc): $c" >&2
    exit $(( rc != 0 ? rc : 99 ))
  fi
done
