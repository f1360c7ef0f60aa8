#!/usr/bin/env python3
"""Randomized ragged batches through the product against the oracle (tooling, GPU box).

    python scripts/fuzz_ragged.py [--batches 60] [--seconds 150] [--uniform 0.25]

Each batch draws a count (4096-300,000), a length distribution (uniform ranges, MTU-sized
mixes, tiny packets, bimodal, 128-B step edges, with zero-length packets), gaps between
packets, overlaps and a base offset 0-15, then checks every checksum against the C oracle
(16 threads).  A share of the batches (--uniform) goes through the uniform entry instead:
back-to-back packets of one 16-B multiple length (the whole-line kernel, with the register
kernel for the head and tail) or of any length and stride.  Stops at the first mismatch and
prints the batch's parameters."""
import argparse
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))


def draw(rng):
    n = int(rng.integers(4096, 300_001))
    kind = int(rng.integers(0, 6))
    if kind == 0:
        lo, hi = sorted(int(x) for x in rng.integers(0, 2000, size=2))
        lengths = rng.integers(lo, hi + 1, size=n)
    elif kind == 1:  # MTU fragments with a short tail every so often
        lengths = np.where(rng.random(n) < 0.05, rng.integers(0, 1392, size=n), 1392)
    elif kind == 2:  # tiny
        lengths = rng.integers(0, 300, size=n)
    elif kind == 3:  # bimodal
        lengths = np.where(rng.random(n) < 0.5, rng.integers(0, 128, size=n), rng.integers(1000, 1800, size=n))
    elif kind == 4:  # 128-B step edges
        lengths = rng.integers(1, 14, size=n) * 128 + rng.integers(-8, 9, size=n)
    else:  # long tail up to 8 KiB
        lengths = np.minimum(rng.exponential(700, size=n).astype(np.int64), 8192)
    lengths = np.clip(lengths, 0, None).astype(np.uint32)
    # zero-length packets: 2 % as a rule, 25 % in some batches (jobs whose first rounds hold only
    # empty packets: no fast body, the generic loop)
    lengths[rng.random(n) < (0.25 if rng.random() < 0.2 else 0.02)] = 0
    gaps = rng.integers(0, 8, size=n) if rng.random() < 0.5 else np.zeros(n, np.int64)
    starts = np.concatenate([[0], np.cumsum(lengths.astype(np.int64) + gaps)[:-1]])
    if rng.random() < 0.2:  # some packets re-read earlier bytes (overlaps are allowed)
        back = rng.integers(0, 64, size=n) * (rng.random(n) < 0.1)
        starts = np.maximum(starts - back, 0)
    base = int(rng.integers(0, 16))
    return kind, base, starts.astype(np.uint64), lengths


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--batches", type=int, default=60)
    ap.add_argument("--seconds", type=float, default=150.0)
    ap.add_argument("--seed", type=int, default=20261017)
    ap.add_argument("--uniform", type=float, default=0.0, help="share of batches through the uniform entry")
    args = ap.parse_args()
    import torch

    import _oracle
    import rusty_enet_amd as rea

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    rng = np.random.default_rng(args.seed)
    t0 = time.time()
    done = packets = 0
    for b in range(args.batches):
        if time.time() - t0 > args.seconds:
            break
        if rng.random() < args.uniform:
            n = int(rng.integers(4096, 300_001))
            if rng.random() < 0.7:  # whole-line shapes: 16-B multiples 528..1792, back to back
                length = int(rng.integers(33, 113)) * 16
                stride, base = length, int(rng.integers(0, 9)) * 16
            else:
                length = int(rng.integers(0, 2100))
                stride, base = length + int(rng.integers(0, 40)), int(rng.integers(0, 16))
            total = (n - 1) * stride + length + base + 8
            data = rng.integers(0, 256, size=total, dtype=np.uint8)
            d = torch.from_numpy(data).to(dev)[base:]
            got = rea.crc32_batch(d, stride=stride, length=length, count=n).cpu().numpy().view(np.uint32)
            want = _oracle.crc32_uniform(data[base:], stride, length, n, threads=16)
            bad = np.flatnonzero(got != want)
            if bad.size:
                print(f"MISMATCH batch {b}: uniform length {length} stride {stride} base +{base} n {n} bad {bad.size}; "
                      f"first packet {int(bad[0])}", flush=True)
                return 1
            done += 1
            packets += n
            print(f"batch {b}: uniform length {length} stride {stride} base +{base} n {n} ok", flush=True)
            continue
        kind, base, starts, lengths = draw(rng)
        total = int((starts + lengths.astype(np.uint64)).max()) + base + 8
        data = rng.integers(0, 256, size=total, dtype=np.uint8)
        d = torch.from_numpy(data).to(dev)[base:]
        off = torch.from_numpy(starts.astype(np.int64)).to(dev)
        ln = torch.from_numpy(lengths.astype(np.int32)).to(dev)
        got = rea.crc32_batch(d, offsets=off, lengths=ln).cpu().numpy().view(np.uint32)
        want = _oracle.crc32_ragged(data[base:], starts, lengths, threads=16)
        bad = np.flatnonzero(got != want)
        if bad.size:
            i = int(bad[0])
            print(f"MISMATCH batch {b}: kind {kind} base +{base} n {lengths.size} bad {bad.size}; first packet {i}: "
                  f"start {int(starts[i])} length {int(lengths[i])}", flush=True)
            return 1
        done += 1
        packets += lengths.size
        print(f"batch {b}: kind {kind} base +{base} n {lengths.size} ok", flush=True)
    print(f"{done} batches, {packets} packets, all bit-exact", flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
