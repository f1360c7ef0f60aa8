#!/usr/bin/env python3
"""Benchmark: device-resident CRC-32 throughput over ENet packet batches (BASELINE.json).

    python bench.py [--gpus N --steps K --warmup W --config uniform|ragged|large|range]

One step = one launch of the batch kernel over this rank's whole shard, inputs
already resident in HBM.  Default workload: 1M x 1200-byte packets on 1 GPU
(BASELINE configs[1]); with N > 1 GPUs each rank takes 2M packets, so N = 8 is
configs[3] (16M x 1200 B sharded 8 ways).  One process per GPU
(torch.distributed.run); shards are independent (no data-path collective), per-GPU
work is fixed as N grows: weak scaling.  Rank 0 prints one JSON line, which at
N = 1 also carries the CPU baseline (oracle on the host cores) and the
end-to-end host->device->host rate of the host-memory entry point.

--config range measures the batched ENet range coder instead:
one step = one compress launch over 1M ragged U{64..1392} compressible packets
(the configs[2] shape); the line also carries the decompress rate and the oracle
(src/c/compress.rs restated in C) timed on one host core.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))

import rusty_enet_amd as rea  # noqa: E402
from rusty_enet_amd.shards import max_over_ranks  # noqa: E402
from _data import ENET_SEED, enet_like_bytes, packed_offsets, ragged_lengths  # noqa: E402

METRIC = "device-resident GiB/s, batched CRC-32 over ENet packets; % HBM3E peak"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec, /opt/skills/guides/MI355X_MICROARCH.md

CONFIGS = {
    # name: (description, packets per GPU at N = 1, packets per GPU at N > 1)
    "uniform": ("1200-byte packets, uniform stride 1200 (ENet batch); BASELINE configs[1] / configs[3]",
                1 << 20, 2 << 20),
    "ragged": ("ragged packets, lengths U{64..1392}, packed at byte offsets; BASELINE configs[2]",
               1 << 20, 1 << 20),
    "large": ("64 KiB buffers, one CRC each (large-buffer path); BASELINE configs[4]", 32768, 32768),
    "range": ("ragged compressible packets, lengths U{64..1392}, range-coder compress (SURVEY.md 8(f)4)",
              1 << 20, 1 << 20),
}
RANGE_METRIC = "device-resident GiB/s, batched ENet range-coder compress (uncompressed input bytes)"
RANGE_WORKERS = 1 << 19  # concurrent coders: 8 waves/SIMD x 4 SIMDs x 64 lanes x 256 CUs (32 GiB arenas)


def packets_per_gpu(name: str, world: int) -> int:
    _, n1, nn = CONFIGS[name]
    return n1 if world == 1 else nn


def make_workload(name: str, rank: int, world: int, dev):
    g = torch.Generator(device=dev)
    g.manual_seed(ENET_SEED + 7919 * rank)
    n = packets_per_gpu(name, world)
    if name == "uniform":
        L = 1200
        data = torch.randint(0, 256, (n * L,), dtype=torch.uint8, device=dev, generator=g)
        out = torch.empty(n, dtype=torch.int32, device=dev)
        step = lambda: rea.crc32_batch(data, stride=L, length=L, count=n, out=out)  # noqa: E731
        return step, n * L, n, out, ("uniform", data, L, L, n)
    if name == "large":
        L = 65536
        data = torch.randint(0, 256, (n * L,), dtype=torch.uint8, device=dev, generator=g)
        out = torch.empty(n, dtype=torch.int32, device=dev)
        step = lambda: rea.crc32_batch(data, stride=L, length=L, count=n, out=out)  # noqa: E731
        return step, n * L, n, out, ("uniform", data, L, L, n)
    lengths = ragged_lengths(ENET_SEED + rank, n)
    offsets = packed_offsets(lengths)
    total = int(lengths.sum())
    if name == "range":
        host = enet_like_bytes(ENET_SEED + rank, total)
        data = torch.from_numpy(host).to(dev)
        off = torch.from_numpy(offsets.astype(np.int64)).to(dev)
        ln = torch.from_numpy(lengths.astype(np.int32)).to(dev)
        res = {}

        def step():
            res["out"] = rea.compress_batch(data, off, ln, workers=RANGE_WORKERS)

        return step, total, n, res, ("range", host, offsets, lengths, data, off, ln)
    data = torch.randint(0, 256, (total,), dtype=torch.uint8, device=dev, generator=g)
    off = torch.from_numpy(offsets.astype(np.int64)).to(dev)
    ln = torch.from_numpy(lengths.astype(np.int32)).to(dev)
    out = torch.empty(n, dtype=torch.int32, device=dev)
    step = lambda: rea.crc32_batch(data, offsets=off, lengths=ln, out=out)  # noqa: E731
    return step, total, n, out, ("ragged", data, offsets, lengths)


def verify_sample(out, spec, limit=20000) -> None:
    """Bit-exact check of a sample of this rank's outputs against the oracle (not timed)."""
    import _oracle

    if spec[0] == "range":
        import _range_oracle as ro

        _, host, offsets, lengths = spec[:4]
        c_out, c_off, c_sizes = out["out"]
        m = min(len(lengths), 4000)
        o_out, o_sizes = ro.compress_ragged(host, offsets[:m], lengths[:m], packed_offsets(lengths[:m]), lengths[:m])
        g_sizes = c_sizes[:m].cpu().numpy().astype(np.uint32)
        g_out, g_off = c_out.cpu().numpy(), c_off[:m].cpu().numpy()
        o_off = packed_offsets(lengths[:m])
        bad = int(np.count_nonzero(g_sizes != o_sizes))
        bad += sum(g_out[int(g_off[p]):int(g_off[p]) + int(g_sizes[p])].tobytes() !=
                   o_out[int(o_off[p]):int(o_off[p]) + int(o_sizes[p])].tobytes() for p in range(m))
        if bad:
            raise SystemExit(f"bench: {bad} of {m} range-coded packets differ from the oracle")
        return
    got = out.cpu().numpy().view(np.uint32)
    if spec[0] == "uniform":
        _, data, stride, length, n = spec
        m = min(n, max(1, limit * 1200 // max(length, 1)))
        host = data[: (m - 1) * stride + length].cpu().numpy()
        want = _oracle.crc32_uniform(host, stride, length, m, threads=8)
    else:
        _, data, offsets, lengths = spec
        m = min(len(lengths), limit)
        end = int(offsets[m - 1]) + int(lengths[m - 1])
        want = _oracle.crc32_ragged(data[:end].cpu().numpy(), offsets[:m], lengths[:m])
    if not np.array_equal(got[:m], want):
        raise SystemExit(f"bench: {int(np.count_nonzero(got[:m] != want))} of {m} checksums differ from the oracle")


def cpu_baseline(seconds: float = 10.0) -> dict:
    """src/crc32.rs restated in C (oracle/), timed on this host: BASELINE configs[0]."""
    import _oracle
    from _data import splitmix64_bytes

    n, L = 4096, 1200
    data = splitmix64_bytes(ENET_SEED, n * L)
    _oracle.crc32_uniform(data, L, L, n)  # warm-up
    times = []
    t_end = time.perf_counter() + seconds
    while time.perf_counter() < t_end or len(times) < 20:
        t0 = time.perf_counter()
        _oracle.crc32_uniform(data, L, L, n)
        times.append(time.perf_counter() - t0)
    single = n * L / float(np.median(times)) / 2**30
    threads = max(1, min(os.cpu_count() or 1, 16))
    mt_times = []
    big = np.tile(data, 8)  # 32768 packets so every thread has work
    t_end = time.perf_counter() + seconds / 4
    while time.perf_counter() < t_end or len(mt_times) < 10:
        t0 = time.perf_counter()
        _oracle.crc32_uniform(big, L, L, 8 * n, threads=threads)
        mt_times.append(time.perf_counter() - t0)
    multi = 8 * n * L / float(np.median(mt_times)) / 2**30
    return {"value": round(single, 4), "unit": "GiB/s", "cores": 1, "kind": "port",
            "sample": f"4096 x 1200 B (BASELINE configs[0]), one crc32 call per packet, median of "
                      f"{len(times)} passes over ~{seconds:.0f} s; C restatement of src/crc32.rs (no rustc here)",
            "all_cores": {"value": round(multi, 4), "cores": threads}}


def range_cpu_baseline(spec, seconds: float = 5.0) -> dict:
    """src/c/compress.rs restated in C (oracle/range_coder_oracle.c) on one host core."""
    import _range_oracle as ro

    _, host, offsets, lengths = spec[:4]
    k = 4096
    nb = int(lengths[:k].sum())
    end = int(offsets[k - 1]) + int(lengths[k - 1])
    times = []
    t_end = time.perf_counter() + seconds
    while time.perf_counter() < t_end or len(times) < 3:
        t0 = time.perf_counter()
        ro.compress_ragged(host[:end], offsets[:k], lengths[:k], packed_offsets(lengths[:k]), lengths[:k])
        times.append(time.perf_counter() - t0)
    return {"value": round(nb / float(np.median(times)) / 2**30, 5), "unit": "GiB/s", "cores": 1, "kind": "port",
            "sample": f"first 4096 packets of the workload ({nb} B), one compress call per packet, median of "
                      f"{len(times)} passes; C restatement of src/c/compress.rs (no rustc here)"}


def range_decompress_rate(spec, res, steps: int = 3) -> dict:
    """Decompress the step's coded packets back (device-resident), timed on the current stream."""
    _, host, offsets, lengths, data, off, ln = spec
    c_out, c_off, c_sizes = res["out"]
    dev = c_out.device
    coded = c_sizes > 0
    idx = torch.nonzero(coded).flatten()
    d_len = c_sizes[idx]
    d_off = c_off[idx]
    lim = ln[idx]
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    out = rea.decompress_batch(c_out, d_off, d_len, lim, workers=RANGE_WORKERS)
    torch.cuda.synchronize()
    ok = bool(torch.equal(out[2][:1000].to(torch.int64), lim[:1000].to(torch.int64)))
    ev0.record()
    for _ in range(steps):
        rea.decompress_batch(c_out, d_off, d_len, lim, workers=RANGE_WORKERS)
    ev1.record()
    torch.cuda.synchronize()
    ms = ev0.elapsed_time(ev1) / steps
    nb = int(lim.to(torch.int64).sum().item())
    return {"value": round(nb / (ms / 1e3) / 2**30, 4), "unit": "GiB/s", "ms": round(ms, 3),
            "packets": int(idx.numel()), "sizes_match_inputs": ok,
            "compressed_fraction": round(float(c_sizes.to(torch.int64).sum().item()) / float(ln.to(torch.int64).sum().item()), 4)}


def end_to_end(dev, n: int = 1 << 18, L: int = 1200) -> dict:
    """Host buffers -> pinned staging -> H2D -> kernel -> D2H (enet_crc32_ragged_host),
    plus the per-call latency of the drop-in hook (enet_crc32_iov, one datagram)."""
    import _oracle
    from _data import splitmix64_bytes

    data = splitmix64_bytes(ENET_SEED + 99, n * L)
    off = np.arange(n, dtype=np.uint64) * np.uint64(L)
    ln = np.full(n, L, dtype=np.uint32)
    ctx = rea.Context(dev.index or 0)
    got = ctx.crc32_ragged_host(data, off, ln)  # warm-up (grows the staging)
    m = 4096
    want = _oracle.crc32_uniform(data[: m * L], L, L, m)
    if not np.array_equal(got[:m], want):
        raise SystemExit("bench: end-to-end checksums differ from the oracle")
    times = []
    for _ in range(5):
        t0 = time.perf_counter()
        ctx.crc32_ragged_host(data, off, ln)
        times.append(time.perf_counter() - t0)
    rate = n * L / float(np.median(times)) / 2**30
    pkt = [data[:1392]]
    for _ in range(50):
        ctx.crc32(pkt)
    t0 = time.perf_counter()
    calls = 2000
    for _ in range(calls):
        ctx.crc32(pkt)
    per_call_us = (time.perf_counter() - t0) / calls * 1e6
    ctx.close()
    return {"value": round(rate, 3), "unit": "GiB/s", "path": "enet_crc32_ragged_host",
            "sample": f"{n} x {L} B from pageable host memory, median of 5 passes",
            "per_call_us": round(per_call_us, 2),
            "per_call_sample": "enet_crc32_iov on one 1392-B datagram (the HostSettings::checksum hook), mean of 2000",
            "ring": ring_rate(dev, L)}


def ring_rate(dev, L: int = 1200, nslots: int = 4, per_slot: int = 40000, rounds: int = 8) -> dict:
    """Pinned receive ring (enet_crc_ring_*): packets already in pinned slot memory,
    H2D + kernel + D2H of each slot on its own stream, slots overlapped."""
    import _oracle
    from _data import splitmix64_bytes
    from rusty_enet_amd.ring import ReceiveRing

    with ReceiveRing(dev.index or 0, nslots=nslots, slot_bytes=per_slot * L, slot_packets=per_slot) as ring:
        for i in range(nslots):
            data, off, ln, _ = ring.slot(i)
            data[:] = splitmix64_bytes(ENET_SEED + 200 + i, per_slot * L)
            off[:] = np.arange(per_slot, dtype=np.uint64) * np.uint64(L)
            ln[:] = L
        for i in range(nslots):
            ring.submit(i, per_slot)
        for i in range(nslots):
            ring.wait(i)
        data, _, _, crcs = ring.slot(0)
        if not np.array_equal(crcs[:1024], _oracle.crc32_uniform(data[:1024 * L].copy(), L, L, 1024)):
            raise SystemExit("bench: ring checksums differ from the oracle")
        t0 = time.perf_counter()
        for _ in range(rounds):
            for i in range(nslots):
                ring.submit(i, per_slot)
            for i in range(nslots):
                ring.wait(i)
        dt = time.perf_counter() - t0
    return {"value": round(rounds * nslots * per_slot * L / dt / 2**30, 3), "unit": "GiB/s",
            "path": "enet_crc_ring_submit/wait",
            "sample": f"{nslots} pinned slots x {per_slot} x {L} B, {rounds} rounds of submit-all/wait-all"}


def load_pmc_traffic(config: str):
    path = os.path.join(REPO, "profiles", "pmc_traffic.json")
    try:
        with open(path) as f:
            v = json.load(f).get(config)
        return None if v is None else v.get("hbm_bytes_per_launch")
    except (OSError, ValueError):
        return None


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=None, help="timed steps (default 200; 5 for --config range)")
    ap.add_argument("--warmup", type=int, default=None, help="untimed steps (default 10; 1 for --config range)")
    ap.add_argument("--config", choices=sorted(CONFIGS), default="uniform")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-verify", action="store_true")
    ap.add_argument("--no-e2e", action="store_true", help="skip the end-to-end host-memory measurement")
    args = ap.parse_args()
    is_range = args.config == "range"
    if args.steps is None:
        args.steps = 5 if is_range else 200
    if args.warmup is None:
        args.warmup = 1 if is_range else 10

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        import torch.distributed as dist

        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    step, nbytes, npk, out, spec = make_workload(args.config, rank, world, dev)
    step()
    torch.cuda.synchronize()
    if not args.no_verify:
        verify_sample(out, spec)
    for _ in range(args.warmup):
        step()

    def barrier():
        if world > 1:
            torch.distributed.barrier()
        torch.cuda.synchronize()

    stream = torch.cuda.current_stream(dev)  # the stream crc32_batch launches on
    ev0 = torch.cuda.Event(enable_timing=True)
    ev1 = torch.cuda.Event(enable_timing=True)
    barrier()
    t0 = time.perf_counter()
    ev0.record(stream)
    for _ in range(args.steps):
        step()
    ev1.record(stream)
    barrier()
    wall = time.perf_counter() - t0
    kernel_ms = ev0.elapsed_time(ev1) / args.steps  # average launch duration on that stream
    wall_max, kernel_ms_max = max_over_ranks([wall, kernel_ms], device=dev)
    ms_per_step = wall_max * 1000.0 / args.steps

    if rank == 0:
        total_bytes = nbytes * world
        value = total_bytes / (ms_per_step / 1000.0) / 2**30
        achieved = nbytes / (kernel_ms / 1000.0) / 1e9  # per-GPU algorithmic GB/s (rank 0)
        traffic = load_pmc_traffic(args.config)
        line = {
            "metric": RANGE_METRIC if is_range else METRIC, "value": round(value, 2), "unit": "GiB/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms_per_step, 5),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u8",
            "data": "synthetic (torch.randint bytes on device, seeded)",
            "config": {"workload": f"{npk} x " + CONFIGS[args.config][0] + " per GPU", "packets_per_gpu": npk,
                       "bytes_per_gpu": nbytes,
                       "parallelism": f"{world} independent shards, no collective"},
            "hbm_frac": round(achieved / HBM_PEAK_GBS, 4),
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                         "kernel_ms": round(kernel_ms, 5), "kernel_ms_max_rank": round(kernel_ms_max, 5)},
        }
        if is_range:
            line["config"]["workers"] = RANGE_WORKERS
            line["data"] = "synthetic compressible ENet-like bytes (tests/_data.enet_like_bytes, seeded)"
            line["roofline"]["note"] = ("latency-bound (dependent arena loads per byte); achieved = "
                                        "uncompressed input bytes per launch / launch time")
            if world == 1:
                line["decompress"] = range_decompress_rate(spec, out)
        if world == 1 and args.cpu_seconds > 0:
            line["cpu_baseline"] = range_cpu_baseline(spec) if is_range else cpu_baseline(args.cpu_seconds)
        if world == 1 and not args.no_e2e and not is_range:
            line["end_to_end"] = end_to_end(dev)
        print(json.dumps(line), flush=True)
    if world > 1:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
