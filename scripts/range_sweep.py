"""Range-coder throughput vs concurrent coders (workers) on one GPU.  Prints one line
per (op, workers): input GiB/s of the batch.  Parity of every packet is checked once
against the oracle on a sample (not timed)."""
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "tests")]
import rusty_enet_amd as rea  # noqa: E402
import _range_oracle as ro  # noqa: E402
from _data import ENET_SEED, enet_like_bytes, packed_offsets, ragged_lengths  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 18
dev = torch.device("cuda:0")
lens = ragged_lengths(ENET_SEED, n)
offs = packed_offsets(lens)
host = enet_like_bytes(ENET_SEED, int(lens.sum()))
data = torch.from_numpy(host).to(dev)
off = torch.from_numpy(offs.astype(np.int64)).to(dev)
ln = torch.from_numpy(lens.astype(np.int32)).to(dev)
nbytes = int(lens.sum())
print(f"packets={n} bytes={nbytes}", flush=True)
out, out_off, sizes = rea.compress_batch(data, off, ln, workers=65536)
torch.cuda.synchronize()
m = 2000
o_out, o_sizes = ro.compress_ragged(host, offs[:m], lens[:m], packed_offsets(lens[:m]), lens[:m])
assert np.array_equal(sizes[:m].cpu().numpy().astype(np.uint32), o_sizes), "compress parity"
csz = sizes.cpu().numpy()
print(f"compressed fraction {csz.sum() / nbytes:.3f}, uncoded packets {int((csz == 0).sum())}", flush=True)
# decompress input: the coded packets
keep = np.nonzero(csz)[0]
oo = out_off.cpu().numpy()
ob = out.cpu().numpy()
c_lens = csz[keep].astype(np.uint32)
c_data = np.concatenate([ob[int(oo[p]):int(oo[p]) + int(csz[p])] for p in keep])
c_offs = packed_offsets(c_lens)
cd = torch.from_numpy(c_data).to(dev)
co = torch.from_numpy(c_offs.astype(np.int64)).to(dev)
cl = torch.from_numpy(c_lens.astype(np.int32)).to(dev)
dl = torch.from_numpy(lens[keep].astype(np.int32)).to(dev)
dec_bytes = int(lens[keep].sum())
for w in [int(x) for x in os.environ.get("SWEEP_WORKERS", "8192 16384 32768 65536 131072 262144").split()]:
    for op in ("compress", "decompress"):
        fn = (lambda: rea.compress_batch(data, off, ln, workers=w)) if op == "compress" else \
             (lambda: rea.decompress_batch(cd, co, cl, dl, workers=w))
        fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        reps = 3
        for _ in range(reps):
            fn()
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / reps
        b = nbytes if op == "compress" else dec_bytes
        print(f"{op:10s} workers={w:7d} {dt * 1e3:9.2f} ms  {b / dt / 2**30:7.3f} GiB/s (uncompressed bytes)", flush=True)
# CPU baseline: oracle compress, one thread, 4096 packets
k = 4096
t0 = time.perf_counter()
ro.compress_ragged(host, offs[:k], lens[:k], packed_offsets(lens[:k]), lens[:k])
dt = time.perf_counter() - t0
print(f"cpu oracle compress 1 thread: {int(lens[:k].sum()) / dt / 2**30:.4f} GiB/s", flush=True)
