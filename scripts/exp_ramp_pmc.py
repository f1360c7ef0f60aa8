#!/usr/bin/env python3
"""G2 launches after an idle gap, for a rocprofv3 --pmc pass (tooling).

    rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE GRBM_UTCL2_BUSY TCP_UTCL1_TRANSLATION_MISS_sum \\
        TCP_UTCL1_TRANSLATION_HIT_sum SQ_BUSY_CYCLES -d <dir> -o run --output-format csv \\
        -- python3 scripts/exp_ramp_pmc.py

One G2 batch (1M x U[64,1392], BASELINE configs[2]) through enet_crc32_ragged_device: 3 s idle,
then `--launches` back-to-back launches.  scripts/ramp_pmc_summary.py pairs each launch's
counters with its duration."""
import argparse
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--launches", type=int, default=200)
    args = ap.parse_args()
    import torch

    import rusty_enet_amd as rea
    from _data import ENET_SEED, packed_offsets, ragged_lengths

    dev = torch.device("cuda", 0)
    lengths = ragged_lengths(ENET_SEED, 1 << 20)
    offsets = packed_offsets(lengths)
    data = torch.randint(0, 256, (int(lengths.sum()),), dtype=torch.uint8, device=dev)
    off = torch.from_numpy(offsets.astype(np.int64)).to(dev)
    ln = torch.from_numpy(lengths.astype(np.int32)).to(dev)
    out = rea.crc32_batch(data, offsets=off, lengths=ln)
    torch.cuda.synchronize()
    time.sleep(3.0)
    for _ in range(args.launches):
        rea.crc32_batch(data, offsets=off, lengths=ln, out=out)
    torch.cuda.synchronize()
    print(f"{args.launches} G2 launches done", flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
