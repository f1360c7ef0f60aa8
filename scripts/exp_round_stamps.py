#!/usr/bin/env python3
"""Experiment (measurement build, make variant NAME=stamps DEFS=-DENET_CRC_ROUND_STAMPS): where
the ragged jobs kernel's waves spend their time -- s_memtime sums per wave of the round
bodies (the slots), the job builds and the whole round loop; the rest is the per-round
bookkeeping (record read and plan, combine, result, flags).  G2, the fragmented 64-KiB
payloads and equal-length ragged batches.
    ENET_CRC_AMD_LIB=rusty_enet_amd/lib/variants/libenet_crc_amd_stamps.so python scripts/exp_round_stamps.py
"""
import ctypes
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))

import rusty_enet_amd as rea  # noqa: E402
from rusty_enet_amd import _native  # noqa: E402
from _data import ENET_SEED, packed_offsets, ragged_lengths  # noqa: E402

f = _native.lib().enet_crc_debug_round_stamps
f.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
buf = (ctypes.c_ulonglong * 8)()
dev = torch.device("cuda:0")
n = 1 << 20
cases = {
    "G2 U[64,1392]": ragged_lengths(ENET_SEED, n),
    "frag 21,845 x 64 KiB": np.tile(np.array([1392] * 48 + [288], dtype=np.uint32), 21845),
    "equal 1200": np.full(n, 1200, dtype=np.uint32),
    "equal 640": np.full(n, 640, dtype=np.uint32),
}
reps = 20
for name, lengths in cases.items():
    off = torch.from_numpy(packed_offsets(lengths).astype(np.int64)).to(dev)
    ln = torch.from_numpy(lengths.astype(np.int32)).to(dev)
    data = torch.randint(0, 256, (int(lengths.sum()),), dtype=torch.uint8, device=dev)
    out = torch.empty(lengths.size, dtype=torch.int32, device=dev)
    run = lambda: rea.crc32_batch(data, offsets=off, lengths=ln, out=out)  # noqa: E731
    run()
    torch.cuda.synchronize()
    assert f(buf, 1) == 0
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        run()
    e1.record()
    e1.synchronize()
    assert f(buf, 1) == 0
    us = e0.elapsed_time(e1) / reps * 1000
    body, loop, rounds, build, comb, make = buf[0], buf[1], buf[2], buf[3], buf[4], buf[5]
    rest = loop - body - build - comb - make
    print(f"{name:22s} {us:8.1f} us/launch  {rounds / reps:9.0f} rounds  per round (cycles): body "
          f"{body / rounds:7.0f}, combine {comb / rounds:6.0f}, plan {make / rounds:6.0f}, builds "
          f"{build / rounds:6.0f}, rest {rest / rounds:6.0f}  (body {100 * body / loop:4.1f} % of the loop)", flush=True)
