#!/bin/bash
# Round 4: the 16-packet ragged kernel: LDS-DMA offset probe, same-process A/B against the
# 8-lane build, the GPU suite, the driver's bench command, instruction counters.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-r04_r16}
mkdir -p $O
timeout -k 5 30 ./tools/lds_dma_offset > $O/lds_dma_offset.txt 2>&1; rc=$?; cat $O/lds_dma_offset.txt; [ $rc = 0 ] || exit $rc
timeout -k 10 150 python -u scripts/ab_ragged.py rusty_enet_amd/lib/libenet_crc_amd.so rusty_enet_amd/lib/variants/libenet_crc_amd_ragged8.so > $O/ab.txt 2>&1 || { cat $O/ab.txt; exit 1; }
grep -v amdgpu.ids $O/ab.txt | grep -v '^{'
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -60 $O/pytest_gpu.log; exit 1; }
tail -3 $O/pytest_gpu.log
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_20_5.json 2> $O/bench_20_5.err || exit $?
python scripts/line_summary.py $O/bench_20_5.json
export TMPDIR=/tmp
for lib in rusty_enet_amd/lib/libenet_crc_amd.so rusty_enet_amd/lib/variants/libenet_crc_amd_ragged8.so; do
  name=$(basename $lib .so)
  for cfg in ragged frag; do
    (cd /tmp && ENET_CRC_AMD_LIB=$GRAFT_REPO_ROOT/$lib timeout -k 10 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES \
      -d $GRAFT_REPO_ROOT/$O/ipc_${name}_$cfg -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --config $cfg --steps 5 --warmup 1 --cpu-seconds 0 --no-verify --no-e2e --no-shard \
      > $GRAFT_REPO_ROOT/$O/ipc_${name}_$cfg.log 2>&1) || exit $?
    python3 scripts/pmc_summary.py $O/ipc_${name}_$cfg > $O/ipc_${name}_${cfg}_summary.txt 2>&1
  done
done
echo "[r16] counters done"
