"""Diagnostic: ragged batches through the product, every mismatch against the oracle printed with
its job, sorted position and round (the job sort and the header rule restated from
crc32_kernels.hip: job_build).  Usage: python scripts/diag_packed.py [count ...]"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
import _oracle  # noqa: E402
from _data import packed_offsets, splitmix64_bytes  # noqa: E402
import rusty_enet_amd as rea  # noqa: E402


def steps(sa, ln):
    z = (4 - (sa + ln) % 4) % 4 if ln else 0
    top, a1 = sa & ~3, (sa + ln + z) & ~3
    nwords = (a1 - top) >> 2
    return ((nwords + 3) // 4 + 7) // 8


def job_packets(count, cus):
    best, jp = None, None
    for rj in range(32, 15, -1):
        p = 8 * rj
        nj = -(-count // p)
        grid = min(nj, cus)
        span = -(-nj // grid) * rj
        if best is None or span < best:
            best, jp = span, p
    return jp


def main():
    dev = torch.device("cuda:0")
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    for count in [int(x) for x in sys.argv[1:]] or [32771]:
        rng = np.random.default_rng(count)
        lengths = rng.integers(0, 3001, size=count).astype(np.uint32)
        lengths[rng.integers(0, count, size=count // 50)] = 0
        gaps = rng.integers(0, 4, size=count).astype(np.uint64)
        offsets = (packed_offsets(lengths) + np.cumsum(gaps)).astype(np.uint64) + np.uint64(3)
        data = splitmix64_bytes(count + 1, int(offsets[-1] + lengths[-1]) + 8)
        d = torch.from_numpy(data).to(dev)
        out = rea.crc32_batch(d, offsets=torch.from_numpy(offsets.astype(np.int64)).to(dev),
                              lengths=torch.from_numpy(lengths.astype(np.int32)).to(dev))
        torch.cuda.synchronize()
        got = out.cpu().numpy().view(np.uint32)
        want = _oracle.crc32_ragged(data, offsets, lengths)
        bad = np.nonzero(got != want)[0]
        JP = job_packets(count, cus)
        print(f"count {count}: JP {JP} mismatches {len(bad)}", flush=True)
        rounds_seen = set()
        for i in bad[:400]:
            J, li = divmod(int(i), JP)
            lo, hi = J * JP, min(count, (J + 1) * JP)
            st = [steps(int(offsets[p]), int(lengths[p])) for p in range(lo, hi)]
            cls = [min(s, 15) for s in st]
            order = sorted(range(hi - lo), key=lambda x: (cls[x], x))
            pos = order.index(li)
            rnd = pos // 8
            if (J, rnd) in rounds_seen:
                continue
            rounds_seen.add((J, rnd))
            members = order[8 * rnd:8 * rnd + 8]
            ms = [st[m] for m in members]
            mx, mn = max(ms), min(ms)
            ns = max(4, (mx + 1) & ~1)
            badm = [m for m in members if got[lo + m] != want[lo + m]]
            print(f"  job {J} round {rnd}/{-(-(hi - lo) // 8)} n={hi - lo} steps {ms} ns {ns} "
                  f"lens {[int(lengths[lo + m]) for m in members]} "
                  f"ends%128 {[int(offsets[lo + m] + lengths[lo + m]) % 128 for m in members]} bad {badm and [members.index(b) for b in badm]}",
                  flush=True)
            if len(rounds_seen) > 40:
                break
    return 0


if __name__ == "__main__":
    sys.exit(main())
