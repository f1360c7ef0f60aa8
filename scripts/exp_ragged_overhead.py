#!/usr/bin/env python3
"""Per-round cost of the ragged machinery: the same bytes through the uniform kernel and
through the ragged path (records pre-pass + round kernel), plus G2.  HIP events on the
stream the launches run on; prints one line per case.  GPU only (an experiment, not a test).

    python scripts/exp_ragged_overhead.py [--reps 50]
"""
from __future__ import annotations

import argparse
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))

import rusty_enet_amd as rea  # noqa: E402
from _data import ENET_SEED, packed_offsets, ragged_lengths  # noqa: E402


def time_it(fn, reps: int) -> float:
    for _ in range(3):
        fn()
    s = torch.cuda.current_stream()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(s)
    for _ in range(reps):
        fn()
    b.record(s)
    b.synchronize()
    return a.elapsed_time(b) / reps * 1000.0  # us


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--only", default="", help="run only the cases whose name contains this")
    ap.add_argument("--lengths", default="", help="comma list: ragged-equal cases at these lengths only")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    n = 1 << 20
    cases = []
    data = torch.randint(0, 256, (n * 1400 + 4096,), dtype=torch.uint8, device=dev)
    out = torch.empty(n, dtype=torch.int32, device=dev)

    def uniform(length):
        return lambda: rea.crc32_batch(data, stride=length, length=length, count=n, out=out)

    def ragged(lengths):
        off = torch.from_numpy(packed_offsets(lengths).astype(np.int64)).to(dev)
        ln = torch.from_numpy(lengths.astype(np.int32)).to(dev)
        return (lambda: rea.crc32_batch(data, offsets=off, lengths=ln, out=out)), int(lengths.sum())

    if args.lengths:
        for length in (int(x) for x in args.lengths.split(",")):
            fn, nb = ragged(np.full(n, length, dtype=np.uint32))
            cases.append((f"ragged-equal {length}", fn, nb))
    for length in (() if args.lengths else (1200, 1392, 640)):
        cases.append((f"uniform {length}", uniform(length), n * length))
        fn, nb = ragged(np.full(n, length, dtype=np.uint32))
        cases.append((f"ragged-equal {length}", fn, nb))
    g2 = ragged_lengths(ENET_SEED, n, lo=64, hi=1392)
    if args.lengths:
        g16 = (g2 + 15) // 16 * 16
        fn, nb = ragged(g16)
        cases.append(("ragged G2 lengths rounded to 16", fn, nb))
    fn, nb = ragged(g2)
    cases.append(("ragged G2 U[64,1392]", fn, nb))
    fn, nb = ragged(np.sort(g2))
    cases.append(("ragged G2 lengths pre-sorted", fn, nb))
    for name, fn, nbytes in cases:
        if args.only not in name:
            continue
        us = time_it(fn, args.reps)
        print(f"{name:32s} {us:9.1f} us  {nbytes / us / 1e3:8.1f} GB/s  frac {nbytes / us / 1e3 / 8000:.3f}",
              flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
