#!/bin/bash
# Round 4: the 16-packet ragged kernel with 128-B loads (ENET_CRC_RAGGED16W build): its
# parity suites, a same-process A/B against the product's 8-lane kernel, and instruction
# counters (with issue-stall split) of both; L2-to-memory read requests of the product's
# ragged and uniform (G1) launches (is FETCH_SIZE x 2 right for partial lines?).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-r04_w}
mkdir -p $O
P=rusty_enet_amd/lib/libenet_crc_amd.so
W=rusty_enet_amd/lib/variants/libenet_crc_amd_ragged16w.so
ENET_CRC_AMD_LIB=$GRAFT_REPO_ROOT/$W timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_slot.py -m gpu -x -v --timeout 240 --timeout-method thread > $O/pytest_gpu_w.log 2>&1 || { tail -40 $O/pytest_gpu_w.log; exit 1; }
tail -2 $O/pytest_gpu_w.log
timeout -k 10 200 python -u scripts/ab_ragged.py $W $P --configs g2,frag > $O/ab_w.txt 2>&1 || { cat $O/ab_w.txt; exit 1; }
grep -v amdgpu.ids $O/ab_w.txt | grep -v '^{'
export TMPDIR=/tmp
for lib in $P $W; do
  name=$(basename $lib .so)
  for cfg in ragged frag; do
    (cd /tmp && ENET_CRC_AMD_LIB=$GRAFT_REPO_ROOT/$lib timeout -k 10 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY \
      -d $GRAFT_REPO_ROOT/$O/ipc_${name}_$cfg -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --config $cfg --steps 5 --warmup 1 --cpu-seconds 0 --no-verify --no-e2e --no-shard \
      > $GRAFT_REPO_ROOT/$O/ipc_${name}_$cfg.log 2>&1) || exit $?
    python3 scripts/pmc_summary.py $O/ipc_${name}_$cfg > $O/ipc_${name}_${cfg}_summary.txt 2>&1
    echo "[w] counters $name $cfg done"
  done
done
for cfg in ragged uniform; do
  (cd /tmp && timeout -s KILL 120 rocprofv3 --kernel-trace --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum \
    -d $GRAFT_REPO_ROOT/$O/rdreq_$cfg -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --config $cfg --steps 5 --warmup 1 --cpu-seconds 0 --no-verify --no-e2e --no-shard \
    > $GRAFT_REPO_ROOT/$O/rdreq_$cfg.log 2>&1) || exit $?
  python3 scripts/pmc_summary.py $O/rdreq_$cfg > $O/rdreq_${cfg}_summary.txt 2>&1
  echo "[w] read requests $cfg done"
done
