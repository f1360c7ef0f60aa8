#!/usr/bin/env python3
"""G1's shape (1M x 1200 B back to back) from bases 0, +16, +48 (head-peeled into the whole-line
kernel) and +8 (register ring), one process, alternating blocks of 20 launches after a
read-ceiling warm-up (tooling).  Prints per-base median kernel us and the fraction of 8 TB/s."""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main() -> int:
    import torch

    import bench
    import rusty_enet_amd as rea

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    n, L = 1 << 20, 1200
    g = torch.Generator(device=dev)
    g.manual_seed(5)
    buf = torch.randint(0, 256, (n * L + 256,), dtype=torch.uint8, device=dev, generator=g)
    assert buf.data_ptr() % 256 == 0
    out = torch.empty(n, dtype=torch.int32, device=dev)
    ceil = bench.open_ceiling(dev)
    if ceil:
        ceil.measure(buf, n * L)
    stream = torch.cuda.current_stream(dev)
    bases = [0, 16, 48, 8]
    times = {b: [] for b in bases}
    for blk in range(6):
        for b in (bases if blk % 2 == 0 else bases[::-1]):
            d = buf[b:b + n * L]
            rea.crc32_batch(d, stride=L, length=L, count=n, out=out)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for _ in range(20):
                rea.crc32_batch(d, stride=L, length=L, count=n, out=out)
            e1.record(stream)
            torch.cuda.synchronize()
            times[b].append(e0.elapsed_time(e1) * 1000.0 / 20)
    for b in bases:
        med = float(np.median(times[b]))
        print(f"base +{b:3d}: median {med:6.1f} us  frac {n * L / (med * 1e-6) / 1e9 / 8000.0:.4f}  "
              f"blocks {[round(t, 1) for t in times[b]]}", flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
