#!/usr/bin/env python3
"""Experiment: where the persistent per-call server is while batch kernels run.  Per-call
latency of a persistent-mode context (1) back to back, (2) after 3 ms of host sleep, (3)
while 20 G2-shaped ragged batches are queued on another stream (the call is made right
after the launches, before they finish), (4) right after those batches finished; and the
batch time with the server resident.
    python scripts/exp_server_latency.py
"""
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))

import rusty_enet_amd as rea  # noqa: E402
from rusty_enet_amd import _native  # noqa: E402
from _data import ENET_SEED, packed_offsets, ragged_lengths  # noqa: E402

dev = torch.device("cuda:0")
n = 1 << 19
lengths = ragged_lengths(ENET_SEED, n)
off = torch.from_numpy(packed_offsets(lengths).astype(np.int64)).to(dev)
ln = torch.from_numpy(lengths.astype(np.int32)).to(dev)
data = torch.randint(0, 256, (int(lengths.sum()),), dtype=torch.uint8, device=dev)
out = torch.empty(n, dtype=torch.int32, device=dev)
batch = lambda: rea.crc32_batch(data, offsets=off, lengths=ln, out=out)  # noqa: E731
batch()
torch.cuda.synchronize()
ctx = rea.Context(0)
ctx.set_percall_mode(_native.ENET_CRC_PERCALL_PERSISTENT)
want = rea.crc32([b"ping"])


def call_us():
    t0 = time.perf_counter()
    got = ctx([b"ping"])
    dt = (time.perf_counter() - t0) * 1e6
    assert got == want
    return dt


for rep in range(3):
    call_us()
    back = [call_us() for _ in range(5)]
    time.sleep(0.003)
    after_sleep = call_us()
    s = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(20):
        batch()
    e1.record(s)
    during = call_us()
    e1.synchronize()
    after_batches = call_us()
    print(f"rep {rep}: back-to-back {np.median(back):6.1f} us, after 3 ms sleep {after_sleep:6.1f} us, "
          f"during batches {during:6.1f} us, after batches {after_batches:6.1f} us, "
          f"batch {e0.elapsed_time(e1) / 20 * 1000:6.1f} us", flush=True)
ctx.close()
