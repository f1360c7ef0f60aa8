#!/usr/bin/env python3
"""Per-launch fixed cost of the batch kernels (tooling).

    python scripts/exp_fixed_overhead.py [libpath] [--reps 3 --launches 20]

Times back-to-back launches of the ragged entry on G2-shaped batches (U[64, 1392] lengths) and
of the uniform entry on G1-shaped batches (1200 B) at 1/16 .. 2 x the headline count, with HIP
events on the launch stream, and fits t(n) = a + b n by least squares over the sizes.  The
intercept a is what a launch costs beyond streaming its bytes: dispatch, the workgroups' start
(table fill, the first job builds), the first loads' latency and the tail.
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("lib", nargs="?", default=os.path.join(REPO, "rusty_enet_amd/lib/libenet_crc_amd.so"))
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--launches", type=int, default=20)
    args = ap.parse_args()

    import torch

    import bench
    from _data import ENET_SEED, packed_offsets, ragged_lengths

    lib = ctypes.CDLL(os.path.abspath(args.lib))
    rag = lib.enet_crc32_ragged_device
    rag.restype = ctypes.c_int
    rag.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p]
    uni = lib.enet_crc32_uniform_device
    uni.restype = ctypes.c_int
    uni.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p]

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    stream = torch.cuda.current_stream(dev)
    ceil = bench.open_ceiling(dev)
    nmax = 1 << 21
    lengths = ragged_lengths(ENET_SEED, nmax)
    offsets = packed_offsets(lengths)
    total = int(lengths.sum())
    g = torch.Generator(device=dev)
    g.manual_seed(ENET_SEED + 12)
    data = torch.randint(0, 256, (max(total, nmax * 1200),), dtype=torch.uint8, device=dev, generator=g)
    off = torch.from_numpy(offsets.astype(np.int64)).to(dev)
    ln = torch.from_numpy(lengths.astype(np.int32)).to(dev)
    out = torch.empty(nmax, dtype=torch.int32, device=dev)
    sizes = [1 << 16, 1 << 17, 1 << 18, 1 << 19, 1 << 20, 1 << 21]
    if ceil:
        ceil.measure(data, total)

    def launch(kind, n):
        if kind == "g2":
            st = rag(data.data_ptr(), off.data_ptr(), ln.data_ptr(), n, out.data_ptr(), stream.cuda_stream)
        else:
            st = uni(data.data_ptr(), 1200, 1200, n, out.data_ptr(), stream.cuda_stream)
        if st != 0:
            raise SystemExit(f"status {st}")

    res = {}
    for kind in ("g2", "g1"):
        t = {n: [] for n in sizes}
        for _ in range(args.reps):
            for n in sizes:
                for _ in range(3):
                    launch(kind, n)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(stream)
                for _ in range(args.launches):
                    launch(kind, n)
                e1.record(stream)
                torch.cuda.synchronize()
                t[n].append(e0.elapsed_time(e1) * 1000.0 / args.launches)
        med = {n: float(np.median(v)) for n, v in t.items()}
        x = np.array(sizes, dtype=np.float64)
        y = np.array([med[n] for n in sizes])
        b, a = np.polyfit(x, y, 1)
        nbytes = {n: (int(lengths[:n].sum()) if kind == "g2" else n * 1200) for n in sizes}
        res[kind] = {"us": {str(n): round(med[n], 2) for n in sizes},
                     "intercept_us": round(float(a), 2), "us_per_Mpacket": round(float(b) * (1 << 20), 2),
                     "bytes": {str(n): nbytes[n] for n in sizes}}
        print(f"{kind}: " + "  ".join(f"{n >> 10}K {med[n]:.1f} us" for n in sizes)
              + f"  -> t = {a:.2f} us + {b * (1 << 20):.2f} us per M packets", flush=True)
    print(json.dumps(res), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
