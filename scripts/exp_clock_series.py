#!/usr/bin/env python3
"""Experiment (measurement build, make variant NAME=clock DEFS=-DENET_CRC_CLOCK_STAMPS): per-launch
time and shader clock of the ragged jobs kernel (G2) and the whole-line kernel (G1) in one
process, from a cold start and after other work (the G2-only 193 -> 150 us
ramp).  Time: HIP events around every launch on its stream.  Clock: the kernel's own
s_memtime / s_memrealtime sums (enet_crc_debug_clock_stamps).  Prints blocks of 10 launches and
one JSON object at the end.  Tooling, not product.

    ENET_CRC_AMD_LIB=rusty_enet_amd/lib/variants/libenet_crc_amd_clock.so python scripts/exp_clock_series.py
"""
from __future__ import annotations

import ctypes
import json
import os
import statistics
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))


def main() -> int:
    import numpy as np
    import torch

    import rusty_enet_amd as rea
    from rusty_enet_amd import _native
    from _data import ENET_SEED, packed_offsets, ragged_lengths

    # The product library has no stamps: then only the times are recorded (the same series
    # run on both builds shows what the stamps themselves cost).
    f = getattr(_native.lib(), "enet_crc_debug_clock_stamps", None)
    if f is not None:
        f.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int, ctypes.POINTER(ctypes.c_uint), ctypes.c_int]
    else:
        f = lambda *a: 0  # noqa: E731
    nslots = 4096
    buf = (ctypes.c_ulonglong * (2 * nslots))()
    launches = ctypes.c_uint(0)

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    stream = torch.cuda.current_stream(dev)
    n = 1 << 20
    g = torch.Generator(device=dev)
    g.manual_seed(1)
    lengths = ragged_lengths(ENET_SEED, n)
    g2_bytes = int(lengths.sum())
    g2 = torch.randint(0, 256, (g2_bytes,), dtype=torch.uint8, device=dev, generator=g)
    off = torch.from_numpy(packed_offsets(lengths).astype(np.int64)).to(dev)
    ln = torch.from_numpy(lengths.astype(np.int32)).to(dev)
    out2 = torch.empty(n, dtype=torch.int32, device=dev)
    g1 = torch.randint(0, 256, (n * 1200,), dtype=torch.uint8, device=dev, generator=g)
    out1 = torch.empty(n, dtype=torch.int32, device=dev)
    import bench

    ceil = bench.ReadCeiling(dev)
    steps = {
        "G2": (lambda: rea.crc32_batch(g2, offsets=off, lengths=ln, out=out2), g2_bytes),
        "G1": (lambda: rea.crc32_batch(g1, stride=1200, length=1200, count=n, out=out1), n * 1200),
        # the same-buffer streaming read (bench.py's ceiling, variant 0): what this box streams
        "ceiling": (lambda: ceil.launch(0, g1, n * 1200), n * 1200),
    }

    def series(name, k):
        fn, nbytes = steps[name]
        torch.cuda.synchronize()
        assert f(buf, 0, ctypes.byref(launches), 1) == 0
        evs = [torch.cuda.Event(enable_timing=True) for _ in range(k + 1)]
        evs[0].record(stream)
        for i in range(k):
            fn()
            evs[i + 1].record(stream)
        torch.cuda.synchronize()
        assert f(buf, k, ctypes.byref(launches), 1) == 0
        stamped = name != "ceiling" and hasattr(_native.lib(), "enet_crc_debug_clock_stamps")
        assert launches.value == (k if stamped else 0), (launches.value, k)
        us = [evs[i].elapsed_time(evs[i + 1]) * 1000.0 for i in range(k)]
        ghz = [buf[2 * i] / buf[2 * i + 1] * 0.1 if stamped and buf[2 * i + 1] else 0.0 for i in range(k)]
        frac = [nbytes / (u * 1e-6) / 8e12 for u in us]
        return {"us": [round(u, 2) for u in us], "ghz": [round(x, 4) for x in ghz], "frac": [round(x, 4) for x in frac]}

    plan = [("idle", 3.0), ("G2", 300), ("G1", 200), ("G2", 100), ("ceiling", 50), ("idle", 3.0), ("G1", 100),
            ("G2", 300), ("idle", 0.5), ("G2", 100), ("ceiling", 50)]
    res = []
    # one launch of each first: code objects loaded, tables built, the fault word registered
    for name in ("G1", "G2"):
        steps[name][0]()
    torch.cuda.synchronize()
    for what, arg in plan:
        if what == "idle":
            time.sleep(arg)
            res.append({"idle_s": arg})
            print(f"-- idle {arg} s", flush=True)
            continue
        r = series(what, arg)
        r["kernel"] = what
        res.append(r)
        print(f"-- {what}: {arg} launches", flush=True)
        for i in range(0, arg, 10):
            u, c = r["us"][i:i + 10], r["ghz"][i:i + 10]
            print(f"{what} {i:4d}-{i + len(u) - 1:4d}: {statistics.fmean(u):7.1f} us (min {min(u):6.1f}, max "
                  f"{max(u):6.1f})  clock {statistics.fmean(c):5.3f} GHz (min {min(c):5.3f}, max {max(c):5.3f})",
                  flush=True)
    out_path = os.environ.get("CLOCK_SERIES_JSON")
    if out_path:
        with open(out_path, "w") as fh:
            json.dump({"device": bench.device_record(dev, 0), "series": res}, fh)
    return 0


if __name__ == "__main__":
    sys.exit(main())
