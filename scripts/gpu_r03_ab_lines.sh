#!/usr/bin/env bash
# A/B of the whole-line G1 kernel (default: register ring, non-temporal loads) against the
# line-split register ring (nolines build) and the whole-line kernel on the LDS-DMA ring
# (linesdma build): full GPU suite on the default build first, then the uniform bench
# config alternating, then rocprof stats, FETCH_SIZE and counters of the default.
#   gpurun --timeout 1200 -- bash scripts/gpu_r03_ab_lines.sh <tag>
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="${1:-r03_lines}"
OUT="$ROOT/gpurun_out/$TAG"
mkdir -p "$OUT"
cd "$ROOT"
V=rusty_enet_amd/lib/variants
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
  --deselect tests/test_gpu_hooks.py::test_batches_next_to_a_persistent_server \
  > "$OUT/pytest_gpu.log" 2>&1 || { tail -40 "$OUT/pytest_gpu.log"; exit 1; }
tail -1 "$OUT/pytest_gpu.log"
bash scripts/gpu_ab_configs.sh "$TAG" none "uniform" 4 rusty_enet_amd/lib/libenet_crc_amd.so \
  $V/libenet_crc_amd_nolines.so $V/libenet_crc_amd_linesdma.so || exit $?
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_uniform" -o run --output-format csv \
  -- python3 "$ROOT/bench.py" --config uniform --steps 20 --warmup 2 --cpu-seconds 0 --no-verify --no-e2e --no-shard \
  > "$OUT/prof_uniform.log" 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d "$OUT/pmc_uniform" -o run --output-format csv \
  -- python3 "$ROOT/bench.py" --config uniform --steps 5 --warmup 1 --cpu-seconds 0 --no-verify --no-e2e --no-shard \
  > "$OUT/pmc_uniform.log" 2>&1 || exit $?
i=0
for counters in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
                "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
                "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --kernel-trace --pmc $counters -d "$OUT/ipc_uniform_$i" -o run --output-format csv \
    -- python3 "$ROOT/bench.py" --config uniform --steps 5 --warmup 1 --cpu-seconds 0 --no-verify --no-e2e --no-shard \
    > "$OUT/ipc_uniform_$i.log" 2>&1 || exit $?
done
cd "$ROOT"
python3 scripts/pmc_summary.py "$OUT"/ipc_uniform_* > "$OUT/ipc_uniform_summary.txt" 2>&1
python3 scripts/pmc_summary.py "$OUT"/pmc_uniform > "$OUT/uniform_pmc_summary.txt" 2>&1
cat "$OUT/prof_uniform/run_kernel_stats.csv" | cut -c1-200 | head -4
cat "$OUT/uniform_pmc_summary.txt" "$OUT/ipc_uniform_summary.txt"
