#!/usr/bin/env python3
"""Packed vs line-aligned datagrams through the product ragged kernel (tooling).

    python scripts/exp_layout.py [--configs g2,frag] [--blocks 12] [--launches 20] [--only packed|aligned]

Same lengths, same payload bytes, two layouts of the batch in HBM: `packed` (datagram i + 1
starts where i ends: neighbours share a 128-B line, the layout every bench line uses) and
`aligned` (every datagram starts on a 128-B boundary: no line holds bytes of two datagrams).
Blocks of launches alternate packed, aligned, ... in one process (HIP events on the launch
stream).  If the shared lines' second read cost load-stream time, the aligned layout would be
faster on the load-bound frag_64k by up to the requests it saves.  Both layouts are checked
against the oracle on a sample.  `--only` runs one layout (for a rocprofv3 --pmc pass)."""
from __future__ import annotations

import argparse
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="g2,frag")
    ap.add_argument("--blocks", type=int, default=12)
    ap.add_argument("--launches", type=int, default=20)
    ap.add_argument("--only", choices=["packed", "aligned"], default=None)
    args = ap.parse_args()

    import torch

    import _oracle
    import bench
    import rusty_enet_amd as rea
    from _data import ENET_SEED, packed_offsets, ragged_lengths

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    stream = torch.cuda.current_stream(dev)
    ceil = bench.open_ceiling(dev)
    layouts = [args.only] if args.only else ["packed", "aligned"]
    res = {}
    for name in args.configs.split(","):
        if name == "g2":
            lengths = ragged_lengths(ENET_SEED, 1 << 20)
        else:
            lengths = np.tile(np.array([1392] * 48 + [288], dtype=np.uint32), 32768)
        n = lengths.size
        payload = int(lengths.sum())
        bufs = {}
        for lay in layouts:
            if lay == "packed":
                offsets = packed_offsets(lengths)
            else:
                stride = (lengths.astype(np.uint64) + 127) // 128 * 128
                offsets = np.concatenate([[0], np.cumsum(stride)[:-1]]).astype(np.uint64)
            total = int(offsets[-1]) + int(lengths[-1])
            g = torch.Generator(device=dev)
            g.manual_seed(ENET_SEED + 11)
            data = torch.randint(0, 256, (total,), dtype=torch.uint8, device=dev, generator=g)
            off = torch.from_numpy(offsets.astype(np.int64)).to(dev)
            ln = torch.from_numpy(lengths.astype(np.int32)).to(dev)
            out = rea.crc32_batch(data, offsets=off, lengths=ln)
            torch.cuda.synchronize()
            m = 50000
            end = int(offsets[m - 1]) + int(lengths[m - 1])
            want = _oracle.crc32_ragged(data[:end].cpu().numpy(), offsets[:m], lengths[:m])
            got = out.cpu().numpy().view(np.uint32)[:m]
            if not np.array_equal(got, want):
                print(json.dumps({name: "MISMATCH", "layout": lay, "n": int(np.count_nonzero(got != want))}))
                return 1
            bufs[lay] = (data, off, ln, out, total)
        if ceil:
            ceil.measure(bufs[layouts[0]][0], bufs[layouts[0]][4])  # through the clock transient
        times = {lay: [] for lay in layouts}
        for blk in range(args.blocks):
            order = layouts if blk % 2 == 0 else layouts[::-1]
            for lay in order:
                data, off, ln, out, _ = bufs[lay]
                rea.crc32_batch(data, offsets=off, lengths=ln, out=out)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(stream)
                for _ in range(args.launches):
                    rea.crc32_batch(data, offsets=off, lengths=ln, out=out)
                e1.record(stream)
                torch.cuda.synchronize()
                times[lay].append(round(e0.elapsed_time(e1) * 1000.0 / args.launches, 2))
        row = {"packets": n, "payload_bytes": payload}
        for lay in layouts:
            med = float(np.median(times[lay]))
            row[lay] = {"us": times[lay], "median_us": med, "footprint_bytes": bufs[lay][4],
                        "frac_payload": round(payload / (med * 1e-6) / 8e12, 4)}
        if len(layouts) == 2:
            row["aligned_vs_packed"] = round(row["aligned"]["median_us"] / row["packed"]["median_us"], 4)
        res[name] = row
        print(name, json.dumps(row), flush=True)
        del bufs
        torch.cuda.empty_cache()
    print(json.dumps(res), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
