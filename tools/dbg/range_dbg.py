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

# per-symbol trace of the debug decoder for the first input
c = ro.compress([b"hello hello hello world"])
src = torch.tensor(list(c), dtype=torch.uint8, device=dev)
out, oo, sizes = rea.decompress_batch(src, torch.zeros(1, dtype=torch.int64, device=dev),
                                      torch.tensor([len(c)], dtype=torch.int32, device=dev),
                                      torch.tensor([8192], dtype=torch.int32, device=dev), workers=1)
t = out.cpu().numpy()[2048:2048 + 16 * 8].view(np.uint32).reshape(8, 4)
for k in range(8):
    w = int(t[k, 0])
    print(k, "v=%c ctx=%u pred=%u low=%08x range=%08x code=%08x" % (w & 0xFF, (w >> 8) & 0xFFF, w >> 20, t[k, 1], t[k, 2], t[k, 3]), flush=True)

a = out.cpu().numpy()[4096:4096 + 256].view(np.uint16).reshape(16, 8)
for k in range(16):
    r = a[k]
    print("sym%2d v=%3u c=%3u u=%5u L=%u R=%u S=%u E=%u T=%u P=%u" % (k, r[0] & 0xFF, r[0] >> 8, r[1], r[2], r[3], r[4], r[5], r[6], r[7]), flush=True)
