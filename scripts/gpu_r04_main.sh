#!/bin/bash
# Round 4: the GPU suite on the product (ragged kernels of both builds), the driver's
# bench command and the default bench, instruction counters of both ragged builds.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-r04_main}
mkdir -p $O
P=rusty_enet_amd/lib/libenet_crc_amd.so
V=rusty_enet_amd/lib/variants
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -60 $O/pytest_gpu.log; exit 1; }
tail -3 $O/pytest_gpu.log
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_20_5.json 2> $O/bench_20_5.err || exit $?
python scripts/line_summary.py $O/bench_20_5.json
timeout -k 10 300 python -u bench.py > $O/bench_default.json 2> $O/bench_default.err || exit $?
python scripts/line_summary.py $O/bench_default.json
export TMPDIR=/tmp
for lib in $P $V/libenet_crc_amd_ragged16.so; do
  name=$(basename $lib .so)
  for cfg in ragged frag; do
    (cd /tmp && ENET_CRC_AMD_LIB=$GRAFT_REPO_ROOT/$lib timeout -k 10 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES \
      -d $GRAFT_REPO_ROOT/$O/ipc_${name}_$cfg -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --config $cfg --steps 5 --warmup 1 --cpu-seconds 0 --no-verify --no-e2e --no-shard \
      > $GRAFT_REPO_ROOT/$O/ipc_${name}_$cfg.log 2>&1) || exit $?
    python3 scripts/pmc_summary.py $O/ipc_${name}_$cfg > $O/ipc_${name}_${cfg}_summary.txt 2>&1
    echo "[main] counters $name $cfg done"
  done
done
