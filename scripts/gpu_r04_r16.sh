#!/bin/bash
# Round 4: the 16-packet ragged kernel: same-process A/B against the 8-lane build, then the
# GPU suite and the driver's bench command.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-r04_r16}
mkdir -p $O
timeout -k 10 300 python -u scripts/ab_ragged.py rusty_enet_amd/lib/libenet_crc_amd.so rusty_enet_amd/lib/variants/libenet_crc_amd_ragged8.so > $O/ab.txt 2>&1 || { cat $O/ab.txt; exit 1; }
grep -v amdgpu.ids $O/ab.txt | grep -v '^{'
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -60 $O/pytest_gpu.log; exit 1; }
tail -3 $O/pytest_gpu.log
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_20_5.json 2> $O/bench_20_5.err || exit $?
python scripts/line_summary.py $O/bench_20_5.json
