#!/bin/bash
# Round 5: randomized ragged batches through the product (256-B pair loads) against the oracle,
# with a new seed.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-r05_fuzz}
mkdir -p $O
timeout -k 10 500 python -u scripts/fuzz_ragged.py --batches 120 --seconds 360 --seed 20261018 > $O/fuzz.txt 2>&1 || { tail -20 $O/fuzz.txt; exit 1; }
tail -3 $O/fuzz.txt
