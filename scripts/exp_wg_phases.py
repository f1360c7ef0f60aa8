#!/usr/bin/env python3
"""Experiment (measurement build libenet_crc_amd_wgstamp3.so, profiles/r06/parked/wg_stamps3.patch:
each workgroup's first wave start, its first wave past the prologue's last barrier, and its last
wave exit; s_memrealtime at 100 MHz; the ragged jobs kernel and the whole-line kernel): how long
a kernel's start (table fill, the first job builds) and its tail take, and whether a workgroup's
start and end follow its index or its XCD.  Tooling, not product.

    ENET_CRC_AMD_LIB=rusty_enet_amd/lib/variants/libenet_crc_amd_wgstamp3.so python scripts/exp_wg_phases.py
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

    f = _native.lib().enet_crc_debug_wg_stamps3
    P = ctypes.POINTER(ctypes.c_ulonglong)
    f.argtypes = [P, P, P, ctypes.c_int, ctypes.c_int]
    dev = torch.device("cuda", 0)
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    g = torch.Generator(device=dev)
    g.manual_seed(1)
    runs = {}
    for name, n in (("G2", 1 << 20), ("G2_64K", 1 << 16)):
        lengths = ragged_lengths(ENET_SEED, n)
        d = torch.randint(0, 256, (int(lengths.sum()),), dtype=torch.uint8, device=dev, generator=g)
        off = torch.from_numpy(packed_offsets(lengths).astype(np.int64)).to(dev)
        ln = torch.from_numpy(lengths.astype(np.int32)).to(dev)
        out = torch.empty(n, dtype=torch.int32, device=dev)
        runs[name] = (lambda d=d, off=off, ln=ln, out=out: rea.crc32_batch(d, offsets=off, lengths=ln, out=out))
    n1 = 1 << 20
    d1 = torch.randint(0, 256, (n1 * 1200,), dtype=torch.uint8, device=dev, generator=g)
    out1 = torch.empty(n1, dtype=torch.int32, device=dev)
    runs["G1"] = lambda: rea.crc32_batch(d1, stride=1200, length=1200, count=n1, out=out1)
    st, mi, en = ((ctypes.c_ulonglong * 4096)() for _ in range(3))
    for name, fn in runs.items():
        for _ in range(30):
            fn()
        torch.cuda.synchronize()
        rows = []
        starts_acc = np.zeros(cus)
        ends_acc = np.zeros(cus)
        for _ in range(40):
            assert f(st, mi, en, 4096, 1) == 0
            fn()
            torch.cuda.synchronize()
            assert f(st, mi, en, 4096, 0) == 0
            s = np.array(st[:cus], dtype=np.float64)
            m = np.array(mi[:cus], dtype=np.float64)
            e = np.array(en[:cus], dtype=np.float64)
            t0 = s.min()
            pro = (m - s) * 0.01
            ends = (e - t0) * 0.01
            rows.append((np.median(pro), pro.max(), (s.max() - t0) * 0.01, ends.max(), ends.max() - np.median(ends),
                         np.median(e - m) * 0.01))
            starts_acc += (s - t0) * 0.01
            ends_acc += ends
        r = np.array(rows)
        if name in ("G2", "G1"):
            sa, ea = starts_acc / 40.0, ends_acc / 40.0
            idx = np.arange(cus)
            print(f"{name} per workgroup (mean of 40 launches): corr(blockIdx, start) {np.corrcoef(idx, sa)[0, 1]:.3f}, "
                  f"corr(blockIdx, end) {np.corrcoef(idx, ea)[0, 1]:.3f}, corr(start, end) {np.corrcoef(sa, ea)[0, 1]:.3f}",
                  flush=True)
            for lo in range(0, cus, cus // 8):
                print(f"  blocks {lo:3d}-{lo + cus // 8 - 1:3d}: start {sa[lo:lo + cus // 8].mean():5.2f} us, "
                      f"end {ea[lo:lo + cus // 8].mean():6.1f} us", flush=True)
            for x in range(8):
                sel = idx % 8 == x
                print(f"  blockIdx % 8 == {x}: start {sa[sel].mean():5.2f} us, end {ea[sel].mean():6.1f} us", flush=True)
        med = [statistics.median(r[:, i]) for i in range(r.shape[1])]
        print(f"{name}: prologue (start -> past the last barrier) median {med[0]:.2f} us, slowest {med[1]:.2f} us; "
              f"start spread {med[2]:.2f} us; first start -> last end {med[3]:.1f} us; last end - median end "
              f"{med[4]:.2f} us; loop time per workgroup median {med[5]:.1f} us", flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
