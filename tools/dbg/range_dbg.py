"""Debug probe: GPU decompress exit reasons (debug build) vs the oracle."""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
import numpy as np, torch
import _range_oracle as ro
import rusty_enet_amd as rea
dev = torch.device("cuda:0")
for x in [b"hello hello hello world", b"a", b"ab"]:
    c = ro.compress([x])
    for lim in (len(x), 8192):
        src = torch.tensor(list(c), dtype=torch.uint8, device=dev)
        offs = torch.zeros(1, dtype=torch.int64, device=dev)
        lens = torch.tensor([len(c)], dtype=torch.int32, device=dev)
        lims = torch.tensor([lim], dtype=torch.int32, device=dev)
        out, oo, sizes = rea.decompress_batch(src, offs, lens, lims, workers=1)
        torch.cuda.synchronize()
        s = int(sizes.cpu()[0]) & 0xFFFFFFFF
        print(x[:12], lim, hex(s), bytes(out.cpu().numpy()[:min(s & 0xFFFF, 32)]), flush=True)

