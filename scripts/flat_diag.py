"""Mismatch diagnostics for the flat ragged kernels (ENET_CRC_RAGGED=flat) on one layout."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
import _oracle  # noqa: E402
from test_gpu_flat import layout, run  # noqa: E402

os.environ["ENET_CRC_RAGGED"] = "flatonly"
dev = torch.device("cuda:0")
for name in sys.argv[1:]:
    data, offsets, lengths = layout(name)
    got = run(data, offsets, lengths, dev)
    want = _oracle.crc32_ragged(data, offsets, lengths)
    bad = np.nonzero(got != want)[0]
    count = len(lengths)
    ngroups = min(32768, max(128, ((count // 2 + 127) // 128) * 128), min(256, (count + 127) // 128) * 128)
    ps = offsets.astype(np.int64)
    pe = ps + lengths.astype(np.int64)
    lo = ps[0] & ~127
    nsteps = ((pe[-1] + 127) & ~127) - lo
    nsteps //= 128
    spg = -(-nsteps // ngroups)
    rb = spg * 128
    cross = (ps - lo) // rb != (np.maximum(pe, ps + 1) - 1 - lo) // rb
    print(f"{name}: count={count} ngroups={ngroups} spg={spg} rb={rb} mismatches={len(bad)} "
          f"crossing={int(cross.sum())} crossing_bad={int(cross[bad].sum()) if len(bad) else 0}")
    for i in bad[:12]:
        r_s, r_e = (ps[i] - lo) // rb, (pe[i] - 1 - lo) // rb
        print(f"  p={i} ps={ps[i]} len={lengths[i]} region {r_s}->{r_e} step_in_region={(ps[i]-lo-r_s*rb)//128}"
              f" end_off_in_step={(pe[i]-lo)%128} idx_in_region_order? got={got[i]:08x} want={want[i]:08x}")
    if len(bad):
        d = np.diff(bad)
        print("  gaps between bad indices (first 20):", d[:20].tolist())
