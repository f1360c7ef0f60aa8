set -e
mkdir -p gpurun_out
timeout -k 10 240 python -u scripts/exp_ragged_overhead.py --lengths 640,641,642,644,648,656,700,704,728,729 > gpurun_out/align_study.txt 2>&1
cat gpurun_out/align_study.txt
