#!/usr/bin/env python3
"""Experiment (measurement build libenet_crc_amd_wgstamp.so: each workgroup's first wave start and
last wave exit, s_memrealtime at 100 MHz, atomicMin / atomicMax into per-workgroup cells): how
long the ragged jobs kernel's last workgroup runs past the others (the static job split's tail).
Tooling, not product.

    ENET_CRC_AMD_LIB=rusty_enet_amd/lib/variants/libenet_crc_amd_wgstamp.so python scripts/exp_wg_tail.py
"""
from __future__ import annotations

import ctypes
import os
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))


def main() -> int:
    import numpy as np
    import torch

    import rusty_enet_amd as rea
    from rusty_enet_amd import _native
    from _data import ENET_SEED, packed_offsets, ragged_lengths

    f = _native.lib().enet_crc_debug_wg_stamps
    f.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int, ctypes.c_int]
    dev = torch.device("cuda", 0)
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    g = torch.Generator(device=dev)
    g.manual_seed(1)
    n = 1 << 20
    lengths = ragged_lengths(ENET_SEED, n)
    g2 = torch.randint(0, 256, (int(lengths.sum()),), dtype=torch.uint8, device=dev, generator=g)
    off = torch.from_numpy(packed_offsets(lengths).astype(np.int64)).to(dev)
    ln = torch.from_numpy(lengths.astype(np.int32)).to(dev)
    out = torch.empty(n, dtype=torch.int32, device=dev)
    # frag_64k: 32,768 payloads of 64 KiB as 49 datagrams each (47 x 1392 + 2 x 288)
    fl = np.tile(np.array([1392] * 47 + [288] * 2, dtype=np.uint32), 32768)
    fb = torch.randint(0, 256, (int(fl.sum()),), dtype=torch.uint8, device=dev, generator=g)
    foff = torch.from_numpy(packed_offsets(fl).astype(np.int64)).to(dev)
    fln = torch.from_numpy(fl.astype(np.int32)).to(dev)
    fout = torch.empty(len(fl), dtype=torch.int32, device=dev)
    runs = {"G2": lambda: rea.crc32_batch(g2, offsets=off, lengths=ln, out=out),
            "frag_64k": lambda: rea.crc32_batch(fb, offsets=foff, lengths=fln, out=fout)}
    st = (ctypes.c_ulonglong * 4096)()
    en = (ctypes.c_ulonglong * 4096)()
    for name, fn in runs.items():
        for _ in range(30):  # warm: clocks up
            fn()
        torch.cuda.synchronize()
        tails, spans, starts, ev_us = [], [], [], []
        for _ in range(40):
            assert f(st, en, 4096, 1) == 0
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            fn()
            e1.record()
            torch.cuda.synchronize()
            assert f(st, en, 4096, 0) == 0
            s = np.array(st[:cus], dtype=np.float64)
            e = np.array(en[:cus], dtype=np.float64)
            t0 = s.min()
            ends = (e - t0) * 0.01  # us
            spans.append(ends.max())
            tails.append(ends.max() - np.median(ends))
            starts.append((s.max() - t0) * 0.01)
            ev_us.append(e0.elapsed_time(e1) * 1000.0)
        print(f"{name}: launch {statistics.median(ev_us):.1f} us (events), first start -> last end "
              f"{statistics.median(spans):.1f} us, last end - median end {statistics.median(tails):.1f} us "
              f"(max {max(tails):.1f}), start spread {statistics.median(starts):.1f} us", flush=True)
        ends_sorted = np.sort(ends)
        print(f"  last launch: workgroup end times (us from first start) p0 {ends_sorted[0]:.1f} p10 "
              f"{ends_sorted[len(ends)//10]:.1f} p50 {ends_sorted[len(ends)//2]:.1f} p90 "
              f"{ends_sorted[9*len(ends)//10]:.1f} p99 {ends_sorted[99*len(ends)//100]:.1f} max {ends_sorted[-1]:.1f}",
              flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
