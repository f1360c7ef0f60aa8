#!/bin/bash
# Instruction counters of the product's ragged kernel (G2 and frag_64k), one rocprofv3 --pmc
# pass each, summarised per launch.   gpurun -- bash scripts/gpu_r06_counters.sh <tag> [lib]
# lib: a variant name (variants/libenet_crc_amd_<name>.so) to count instead of the product.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
if [ -n "$2" ]; then export ENET_CRC_AMD_LIB=$PWD/rusty_enet_amd/lib/variants/libenet_crc_amd_$2.so; fi
for c in ragged frag; do
  timeout -k 10 120 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS \
    -d "$O/ipc_$c" -o run --output-format csv \
    -- python3 bench.py --config $c --steps 5 --warmup 1 --cpu-seconds 0 --no-verify --no-e2e --no-shard \
    > "$O/ipc_$c.log" 2>&1 || exit $?
  python3 scripts/pmc_summary.py "$O/ipc_$c" > "$O/ipc_${c}_summary.txt" 2>&1
  grep -E "INSTS_(VALU|SALU|LDS)" "$O/ipc_${c}_summary.txt" | sed "s/^/$c /"
done
echo "[counters] done"
