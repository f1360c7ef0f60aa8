#!/bin/bash
# The driver's N = 2 / 4 bench command rehearsed on the one GPU (ranks share it,
# BENCH_SHARE_GPUS=1); stdout must be exactly rank 0's JSON line.
#   gpurun -- bash scripts/gpu_r06_rehearsal.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/$1
mkdir -p $O
for n in 2 4; do
  BENCH_SHARE_GPUS=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n \
    --master-addr 127.0.0.1 --master-port $((29500 + n)) bench.py --gpus $n --steps 20 --warmup 5 \
    > $O/bench_rehearsal_n$n.json 2> $O/bench_rehearsal_n$n.err || { tail -20 $O/bench_rehearsal_n$n.err; exit 1; }
  python -c "import json,sys; t=open('$O/bench_rehearsal_n$n.json').read().strip().splitlines(); assert len(t)==1, t; d=json.loads(t[0]); print($n, d['value'], d['unit'], d['n_gpus'])" || exit 1
done
echo "[rehearsal] done"
