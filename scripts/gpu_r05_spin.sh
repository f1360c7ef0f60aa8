#!/bin/bash
# How long the ragged kernel's waves spin on LDS flags (ENET_CRC_SPIN_STAMPS build).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-r05_spin}
mkdir -p $O
timeout -k 10 300 python -u scripts/exp_spin.py rusty_enet_amd/lib/variants/libenet_crc_amd_spin.so > $O/spin.txt 2>&1 || { tail -20 $O/spin.txt; exit 1; }
cat $O/spin.txt
