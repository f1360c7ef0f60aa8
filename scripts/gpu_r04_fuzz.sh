#!/bin/bash
# Round 4: randomized ragged batches through the product against the oracle.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-r04_fuzz}
mkdir -p $O
timeout -k 10 400 python -u scripts/fuzz_ragged.py --batches 80 --seconds 240 > $O/fuzz.txt 2>&1 || { tail -20 $O/fuzz.txt; exit 1; }
tail -3 $O/fuzz.txt
