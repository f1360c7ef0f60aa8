#!/bin/bash
# Round 6: randomized ragged batches through the product against the oracle, with a new seed.
#   gpurun -- bash scripts/gpu_r06_fuzz.sh <tag> [seed] [share of uniform batches]
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-r06_fuzz}
mkdir -p $O
timeout -k 10 500 python -u scripts/fuzz_ragged.py --batches 160 --seconds 380 --uniform ${3:-0} --seed ${2:-20261019} > $O/fuzz.txt 2>&1 || { tail -20 $O/fuzz.txt; exit 1; }
tail -3 $O/fuzz.txt
