#!/usr/bin/env python3
"""Experiment: how G1's launch time and the same-buffer read ceiling move within one
process (idle -> burst, sustained, alternating).  Per-launch HIP event times on the
launch stream; prints one JSON object.  Tooling, not product."""
from __future__ import annotations

import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))


def main() -> int:
    import torch

    import bench
    import rusty_enet_amd as rea

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    n, L = 1 << 20, 1200
    g = torch.Generator(device=dev)
    g.manual_seed(1)
    data = torch.randint(0, 256, (n * L,), dtype=torch.uint8, device=dev, generator=g)
    out = torch.empty(n, dtype=torch.int32, device=dev)
    step = lambda: rea.crc32_batch(data, stride=L, length=L, count=n, out=out)  # noqa: E731
    ceil = bench.ReadCeiling(dev)
    stream = torch.cuda.current_stream(dev)

    def series(fn, k):
        evs = [torch.cuda.Event(enable_timing=True) for _ in range(k + 1)]
        evs[0].record(stream)
        for i in range(k):
            fn()
            evs[i + 1].record(stream)
        torch.cuda.synchronize()
        return [round(evs[i].elapsed_time(evs[i + 1]) * 1000.0, 1) for i in range(k)]

    res = {}
    step()
    torch.cuda.synchronize()
    time.sleep(3.0)
    res["A_burst_warm5"] = series(step, 5)
    res["A_burst_timed20"] = series(step, 20)
    res["B_sustained200"] = series(step, 200)
    for v in range(ceil.variants):
        res[f"C_ceiling_v{v}_{ceil.name(v)}"] = series(lambda v=v: ceil.launch(v, data, n * L), 20)
    time.sleep(3.0)
    res["D_ceiling_v0_after_idle"] = series(lambda: ceil.launch(0, data, n * L), 25)
    res["D_g1_after_ceiling"] = series(step, 25)
    time.sleep(3.0)
    alt = series(lambda: (step(), ceil.launch(0, data, n * L)), 20)
    res["E_alternating_pairs"] = alt
    print(json.dumps(res), flush=True)
    for k, v in res.items():
        s = sorted(v)
        print(f"{k:40s} n={len(v):3d} first={v[0]:7.1f} min={s[0]:7.1f} med={s[len(s)//2]:7.1f} "
              f"max={s[-1]:7.1f} mean={sum(v)/len(v):7.1f}", flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
