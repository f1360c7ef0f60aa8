"""Experiment (test-hooks build): G2-shaped ragged batch time with and without a resident
persistent server wave and with 0 or 8 CUs held back (ENET_CRC_TEST_RESERVE), cases
interleaved and repeated.  Only the launch stream is synchronised: a device-wide
synchronize would wait for the server to exit (its 20-ms idle limit).
    ENET_CRC_AMD_LIB=rusty_enet_amd/lib/variants/libenet_crc_amd_testhooks.so python scripts/exp_server_overlap.py"""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
from _data import ENET_SEED, packed_offsets, ragged_lengths  # noqa: E402

import rusty_enet_amd as rea  # noqa: E402
from rusty_enet_amd import _native  # noqa: E402

dev = torch.device("cuda:0")
ctx = rea.Context(0)
ctx.set_percall_mode(_native.ENET_CRC_PERCALL_PERSISTENT)
for n in (1 << 19, 1 << 20):
    lengths = ragged_lengths(ENET_SEED, n)
    offsets = packed_offsets(lengths)
    data = torch.randint(0, 256, (int(lengths.sum()),), dtype=torch.uint8, device=dev)
    off = torch.from_numpy(offsets.astype(np.int64)).to(dev)
    ln = torch.from_numpy(lengths.astype(np.int32)).to(dev)
    out = torch.empty(n, dtype=torch.int32, device=dev)

    def timed(reps=20):
        rea.crc32_batch(data, offsets=off, lengths=ln, out=out)
        torch.cuda.current_stream().synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            rea.crc32_batch(data, offsets=off, lengths=ln, out=out)
        e1.record()
        e1.synchronize()
        return e0.elapsed_time(e1) / reps * 1000

    for rep in range(3):
        for server in (False, True):
            for rsv in ("0", "1", "8"):
                os.environ["ENET_CRC_TEST_RESERVE"] = rsv
                if server:
                    assert ctx([b"x"]) == rea.crc32([b"x"])  # resident from here
                else:
                    ctx.stop_server()
                t = timed()
                c0 = time.perf_counter()
                if server:
                    got = ctx([b"y"])
                call_us = (time.perf_counter() - c0) * 1e6
                if server:
                    assert got == rea.crc32([b"y"])
                # a resident server answers in a few us; a relaunch after it exited costs ~20 us
                print(f"n={n} rep={rep} server={'live' if server else 'none':4s} {rsv} CUs held back {t:8.1f} us"
                      f"  next call {call_us:6.1f} us", flush=True)
os.environ.pop("ENET_CRC_TEST_RESERVE")
ctx.close()
