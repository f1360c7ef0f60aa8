#!/bin/bash
# Round 6's evidence on its final sources: the GPU suite, smoke(), the driver's bench command,
# the driver's N = 2 / 4 command rehearsed on the one GPU (ranks share it, BENCH_SHARE_GPUS=1),
# then the profile round (kernel stats, FETCH_SIZE, read sizes, counters, traces).
#   gpurun --timeout 1200 -- bash scripts/gpu_r06_final.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
T=${1:-r06_final}
O=gpurun_out/$T
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -60 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_20_5.json 2> $O/bench_20_5.err || exit $?
python scripts/line_summary.py $O/bench_20_5.json
for n in 2 4; do
  BENCH_SHARE_GPUS=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n \
    --master-addr 127.0.0.1 --master-port $((29500 + n)) bench.py --gpus $n --steps 20 --warmup 5 \
    > $O/bench_rehearsal_n$n.json 2> $O/bench_rehearsal_n$n.err || { tail -20 $O/bench_rehearsal_n$n.err; exit 1; }
  echo "[final] rehearsal N=$n done"
done
bash scripts/gpu_profile_round.sh $T || exit $?
python scripts/line_summary.py $O/bench_uniform.json
echo "[final] done"
