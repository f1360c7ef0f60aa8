"""G2 (1M x U[64,1392] packed) through ENET_CRC_RAGGED=flat and =sorted vs the oracle."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
import _oracle  # noqa: E402
from _data import ENET_SEED, packed_offsets, ragged_lengths  # noqa: E402
import rusty_enet_amd as rea  # noqa: E402

dev = torch.device("cuda:0")
n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 20
lengths = ragged_lengths(ENET_SEED, n)
offsets = packed_offsets(lengths)
g = torch.Generator(device=dev)
g.manual_seed(ENET_SEED + 9)
d = torch.randint(0, 256, (int(lengths.sum()),), dtype=torch.uint8, device=dev, generator=g)
off = torch.from_numpy(offsets.astype(np.int64)).to(dev)
ln = torch.from_numpy(lengths.astype(np.int32)).to(dev)
want = _oracle.crc32_ragged(d.cpu().numpy(), offsets, lengths)
ps = offsets.astype(np.int64)
pe = ps + lengths.astype(np.int64)
ngroups = 32768
nsteps = (((pe[-1] + 127) & ~127) - (ps[0] & ~127)) // 128
rb = -(-nsteps // ngroups) * 128
for mode in ["flatonly", "sorted", "flat", "default"]:
    if mode == "default":
        os.environ.pop("ENET_CRC_RAGGED", None)
    else:
        os.environ["ENET_CRC_RAGGED"] = mode
    got = rea.crc32_batch(d, offsets=off, lengths=ln)
    torch.cuda.synchronize()
    got = got.cpu().numpy().view(np.uint32)
    bad = np.nonzero(got != want)[0]
    print(f"{mode}: mismatches={len(bad)} rb={rb}", flush=True)
    for i in bad[:10]:
        rs, re_ = ps[i] // rb, (pe[i] - 1) // rb
        # packet index within its emitting region
        first_in_region = np.searchsorted(pe, re_ * rb, side="right")
        print(f"  p={i} ps={ps[i]} len={lengths[i]} regions {rs}->{re_} ps%128={ps[i] % 128} "
              f"pe%128={pe[i] % 128} k_in_region={i - first_in_region} got={got[i]:08x} want={want[i]:08x}")
