#!/bin/bash
# Round-5 bound probes: ablation A/Bs (product = A) and read requests of the product and of
# one variant on G2 (over-fetch).   gpurun -- bash scripts/gpu_r05_probe.sh <tag> <rdreq-variant> <ablation>...
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
TAG=$1; RV=$2; shift 2
O=gpurun_out/$TAG
mkdir -p $O
bash scripts/gpu_r05_abl.sh $TAG g2,frag,r740 "$@" || exit 1
export TMPDIR=/tmp
for L in product $RV; do
  if [ $L = product ]; then unset ENET_CRC_AMD_LIB; else export ENET_CRC_AMD_LIB=$GRAFT_REPO_ROOT/rusty_enet_amd/lib/variants/libenet_crc_amd_$L.so; fi
  (cd /tmp && timeout -s KILL 120 rocprofv3 --kernel-trace --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum \
    -d "$GRAFT_REPO_ROOT/$O/rdreq_$L" -o run --output-format csv \
    -- python3 "$GRAFT_REPO_ROOT/bench.py" --config ragged --steps 5 --warmup 1 --cpu-seconds 0 --no-verify --no-e2e --no-shard \
    > "$GRAFT_REPO_ROOT/$O/rdreq_$L.log" 2>&1) || exit 1
  python3 scripts/pmc_summary.py "$O/rdreq_$L" > "$O/rdreq_${L}_summary.txt" 2>&1
  echo "== rdreq $L"; cat "$O/rdreq_${L}_summary.txt"
done
echo "[probe] done"
