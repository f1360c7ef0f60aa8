#!/usr/bin/env python3
"""Same-process alternating A/B of two builds of the library on ragged batches (tooling).

    python scripts/ab_ragged.py libA.so libB.so [--blocks 6 --launches 20]

Both builds are loaded side by side (ctypes, RTLD_LOCAL: each keeps its own kernels) and
called through enet_crc32_ragged_device on the same device buffers: G2 (1M x U[64,1392],
BASELINE configs[2]) and frag_64k (32,768 x 64 KiB payloads as 49 datagrams each); rNNN = 1M datagrams of NNN
bytes through the ragged entry; g1 / mtu through the uniform entry.  Both
outputs are checked against each other in full and against the oracle on a sample; then
blocks of `launches` back-to-back launches alternate A, B, A, B, ... after a read-ceiling
warm-up, timed with HIP events on the launch stream.  Prints per-block kernel us and the
roofline fraction of 8 TB/s."""
from __future__ import annotations

import argparse
import ctypes
import time
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))


def load(path: str):
    lib = ctypes.CDLL(os.path.abspath(path))
    f = lib.enet_crc32_ragged_device
    f.restype = ctypes.c_int
    f.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p]
    u = lib.enet_crc32_uniform_device
    u.restype = ctypes.c_int
    u.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p]
    return f, u


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("a")
    ap.add_argument("b")
    ap.add_argument("--blocks", type=int, default=6)
    ap.add_argument("--launches", type=int, default=20)
    ap.add_argument("--configs", default="g2,frag")
    ap.add_argument("--unchecked-b", action="store_true", help="B is a measurement build: do not compare its output")
    ap.add_argument("--cold", type=float, default=0.0,
                    help="idle this many seconds before each block (then 5 untimed launches): the cold window")
    args = ap.parse_args()

    import torch

    import _oracle
    import bench
    from _data import ENET_SEED, packed_offsets, ragged_lengths

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    (fa, ua), (fb, ub) = load(args.a), load(args.b)
    stream = torch.cuda.current_stream(dev)
    ceil = bench.open_ceiling(dev)
    res = {}
    for name in args.configs.split(","):
        uniform = name in ("g1", "mtu")
        if name == "g2":
            lengths = ragged_lengths(ENET_SEED, 1 << 20)
        elif name.startswith("r") and name[1:].isdigit():  # ragged API, one length (e.g. r740)
            lengths = np.full(1 << 20, int(name[1:]), dtype=np.uint32)
        elif uniform:
            lengths = np.full(1 << 20, 1200 if name == "g1" else 1392, dtype=np.uint32)
        else:
            lengths = np.tile(np.array([1392] * 48 + [288], dtype=np.uint32), 32768)
        offsets = packed_offsets(lengths)
        total = int(lengths.sum())
        g = torch.Generator(device=dev)
        g.manual_seed(ENET_SEED + 11)
        data = torch.randint(0, 256, (total,), dtype=torch.uint8, device=dev, generator=g)
        off = torch.from_numpy(offsets.astype(np.int64)).to(dev)
        ln = torch.from_numpy(lengths.astype(np.int32)).to(dev)
        oa = torch.empty(lengths.size, dtype=torch.int32, device=dev)
        ob = torch.empty(lengths.size, dtype=torch.int32, device=dev)
        n = lengths.size

        L0 = int(lengths[0])

        def run(f, out):
            if uniform:
                u = ua if f is fa else ub
                st = u(data.data_ptr(), L0, L0, n, out.data_ptr(), stream.cuda_stream)
            else:
                st = f(data.data_ptr(), off.data_ptr(), ln.data_ptr(), n, out.data_ptr(), stream.cuda_stream)
            if st != 0:
                raise SystemExit(f"status {st}")

        run(fa, oa)
        run(fb, ob)
        torch.cuda.synchronize()
        ga, gb = oa.cpu().numpy().view(np.uint32), ob.cpu().numpy().view(np.uint32)
        m = 50000
        end = int(offsets[m - 1]) + int(lengths[m - 1])
        want = _oracle.crc32_ragged(data[:end].cpu().numpy(), offsets[:m], lengths[:m])
        ok = (args.unchecked_b or bool(np.array_equal(ga, gb))) and bool(np.array_equal(ga[:m], want))
        if not ok:
            print(json.dumps({name: "MISMATCH", "a_vs_b": int(np.count_nonzero(ga != gb)),
                              "a_vs_oracle": int(np.count_nonzero(ga[:m] != want)),
                              "b_vs_oracle": int(np.count_nonzero(gb[:m] != want))}), flush=True)
            return 1
        if ceil:
            ceil.measure(data, total)  # warm-up through the power-management transient
        times = {"a": [], "b": []}
        for blk in range(args.blocks):
            for key, f, out in (("a", fa, oa), ("b", fb, ob)) if blk % 2 == 0 else (("b", fb, ob), ("a", fa, oa)):
                if args.cold > 0:
                    torch.cuda.synchronize()
                    time.sleep(args.cold)
                    for _ in range(4):
                        run(f, out)
                run(f, out)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(stream)
                for _ in range(args.launches):
                    run(f, out)
                e1.record(stream)
                torch.cuda.synchronize()
                times[key].append(round(e0.elapsed_time(e1) * 1000.0 / args.launches, 2))
        frac = {k: [round(total / (t * 1e-6) / 1e9 / 8000.0, 4) for t in v] for k, v in times.items()}
        res[name] = {"bytes": total, "packets": n, "us": times, "frac": frac,
                     "a_median_us": float(np.median(times["a"])), "b_median_us": float(np.median(times["b"]))}
        print(f"{name}: A {times['a']} us  B {times['b']} us  -> median A {res[name]['a_median_us']:.1f} "
              f"B {res[name]['b_median_us']:.1f} (frac A {max(frac['a'])}-{min(frac['a'])}, "
              f"B {max(frac['b'])}-{min(frac['b'])})", flush=True)
        del data, off, ln, oa, ob
        torch.cuda.empty_cache()
    print(json.dumps({"a": args.a, "b": args.b, **res}), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
