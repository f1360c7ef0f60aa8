#!/bin/bash
# Round 4: LDS-DMA offset probe; the 16-packet ragged kernel (ENET_CRC_RAGGED16 build)
# against the product's 8-lane kernel in one process; where G1's time goes (measurement
# builds); the GPU suite on the product and the parity suites on the ragged16 build; the
# driver's bench command; instruction counters of both ragged kernels.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-r04_r16}
mkdir -p $O
P=rusty_enet_amd/lib/libenet_crc_amd.so
V=rusty_enet_amd/lib/variants
timeout -k 5 30 ./tools/lds_dma_offset > $O/lds_dma_offset.txt 2>&1; rc=$?; cat $O/lds_dma_offset.txt; [ $rc = 0 ] || exit $rc
timeout -k 10 150 python -u scripts/ab_ragged.py $V/libenet_crc_amd_ragged16.so $P > $O/ab.txt 2>&1 || { cat $O/ab.txt; exit 1; }
grep -v amdgpu.ids $O/ab.txt | grep -v '^{'
for v in g1nocombine g1nolookups; do
  timeout -k 10 150 python -u scripts/ab_ragged.py $P $V/libenet_crc_amd_$v.so --configs g1 --unchecked-b > $O/ab_$v.txt 2>&1 || { cat $O/ab_$v.txt; exit 1; }
  grep -v amdgpu.ids $O/ab_$v.txt | grep -v '^{'
done
ENET_CRC_AMD_LIB=$GRAFT_REPO_ROOT/$V/libenet_crc_amd_ragged16.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_slot.py -m gpu -x -v --timeout 240 --timeout-method thread > $O/pytest_gpu_ragged16.log 2>&1 || { tail -40 $O/pytest_gpu_ragged16.log; exit 1; }
tail -2 $O/pytest_gpu_ragged16.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -60 $O/pytest_gpu.log; exit 1; }
tail -3 $O/pytest_gpu.log
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_20_5.json 2> $O/bench_20_5.err || exit $?
python scripts/line_summary.py $O/bench_20_5.json
export TMPDIR=/tmp
for lib in $P $V/libenet_crc_amd_ragged16.so; do
  name=$(basename $lib .so)
  for cfg in ragged frag; do
    (cd /tmp && ENET_CRC_AMD_LIB=$GRAFT_REPO_ROOT/$lib timeout -k 10 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES \
      -d $GRAFT_REPO_ROOT/$O/ipc_${name}_$cfg -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --config $cfg --steps 5 --warmup 1 --cpu-seconds 0 --no-verify --no-e2e --no-shard \
      > $GRAFT_REPO_ROOT/$O/ipc_${name}_$cfg.log 2>&1) || exit $?
    python3 scripts/pmc_summary.py $O/ipc_${name}_$cfg > $O/ipc_${name}_${cfg}_summary.txt 2>&1
  done
done
echo "[r16] counters done"
