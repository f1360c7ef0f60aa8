#!/usr/bin/env python3
"""Benchmark: device-resident CRC-32 throughput over ENet packet batches (BASELINE.json).

    python bench.py [--gpus N --steps K --warmup W --config uniform|ragged|large|range]

One step = one launch of the batch kernel over this rank's whole shard, inputs
already resident in HBM.  Default workload: 1M x 1200-byte packets on 1 GPU
(BASELINE configs[1]); with N > 1 GPUs each rank takes 2M packets, so N = 8 is
configs[3] (16M x 1200 B sharded 8 ways).  At N = 1 the line also times the same
2M-packet shard (``shard_2m``), so the per-GPU work behind the N = 1 and N > 1
numbers can be compared like for like.

Multi-GPU: one process per GPU.  ``--gpus N`` without an enclosing torchrun
starts ``torch.distributed.run`` with N ranks as a child process (before anything
touches the GPU) and exits with its status; under torchrun, ``--gpus`` must equal
WORLD_SIZE.  Shards are independent (no data-path collective); the max-over-ranks
timing uses a gloo process group on the CPU.  Per-GPU work is fixed as N grows:
weak scaling.  Rank 0 prints one JSON line, which at N = 1 also carries the CPU
baseline (oracle on the host cores) and the end-to-end host->device->host rates.

--config range measures the batched ENet range coder instead:
one step = one compress launch over 1M ragged U{64..1392} compressible packets
(the configs[2] shape); the line also carries the decompress rate and the oracle
(src/c/compress.rs restated in C) timed on one host core.
"""
from __future__ import annotations

import argparse
import hashlib
import json
import math
import os
import socket
import subprocess
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))

METRIC = "device-resident GiB/s, batched CRC-32 over ENet packets; % HBM3E peak"
RANGE_METRIC = "device-resident GiB/s, batched ENet range-coder compress (uncompressed input bytes)"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec, /opt/skills/guides/MI355X_MICROARCH.md
RANGE_WORKERS = 1 << 18  # concurrent range coders (16 GiB of arenas; 512K coders measured no faster)

CONFIGS = {
    # name: (description, packets per GPU at N = 1, packets per GPU at N > 1)
    "uniform": ("1200-byte packets, uniform stride 1200 (ENet batch); BASELINE configs[1] / configs[3]",
                1 << 20, 2 << 20),
    "ragged": ("ragged packets, lengths U{64..1392}, packed at byte offsets; BASELINE configs[2]",
               1 << 20, 1 << 20),
    "large": ("64 KiB buffers, one CRC each (large-buffer path); BASELINE configs[4]", 32768, 32768),
    "frag": ("64 KiB payloads fragmented at the default MTU (48 x 1392 B + 288 B datagrams each, one CRC per "
             "datagram); the configs[4] bytes as the reference checksums them", 32768, 32768),
    "range": ("ragged compressible packets, lengths U{64..1392}, range-coder compress (SURVEY.md 8(f)4)",
              1 << 20, 1 << 20),
}
# Source files whose change invalidates a committed traffic measurement.
KERNEL_SOURCES = ("crc32_kernels.hip", "crc32_geometry.hpp", "crc32_layout.hpp", "crc32_ops.hpp",
                  "crc32_kernels.hpp", "range_coder.hip", "range_coder.hpp")


def packets_per_gpu(name: str, world: int, override: int | None = None) -> int:
    if override:
        return override
    _, n1, nn = CONFIGS[name]
    return n1 if world == 1 else nn


# --------------------------------------------------------------------------------------
# multi-process launch
# --------------------------------------------------------------------------------------

def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn_command(gpus: int, argv: list[str], port: int) -> list[str]:
    """torch.distributed.run command that re-runs this script with `gpus` ranks."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={gpus}",
            "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__), *argv]


def visible_gpus() -> int:
    import torch

    return torch.cuda.device_count()  # does not initialise the GPU on this image


def spawn(args, argv: list[str]) -> int:
    """Start N ranks as a child process group (nothing here has touched the GPU)."""
    have = visible_gpus()
    # BENCH_SHARE_GPUS=1 (rehearsal only): ranks share the visible GPUs round-robin, so the
    # multi-process path can be exercised on a 1-GPU box.  The line then says so.
    if have < args.gpus and not (os.environ.get("BENCH_SHARE_GPUS") == "1" and have > 0):
        print(f"bench: --gpus {args.gpus} requested but only {have} HIP device(s) are visible",
              file=sys.stderr, flush=True)
        return 2
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    return subprocess.call(spawn_command(args.gpus, argv, _free_port()), env=env)


# --------------------------------------------------------------------------------------
# workloads
# --------------------------------------------------------------------------------------

def make_workload(name: str, rank: int, n: int, dev, length: int | None = None):
    import torch

    import rusty_enet_amd as rea
    from _data import ENET_SEED, enet_like_bytes, packed_offsets, ragged_lengths

    g = torch.Generator(device=dev)
    g.manual_seed(ENET_SEED + 7919 * rank)
    if name in ("uniform", "large"):
        L = length or (1200 if name == "uniform" else 65536)
        data = torch.randint(0, 256, (n * L,), dtype=torch.uint8, device=dev, generator=g)
        out = torch.empty(n, dtype=torch.int32, device=dev)
        step = lambda: rea.crc32_batch(data, stride=L, length=L, count=n, out=out)  # noqa: E731
        return step, n * L, n, out, ("uniform", data, L, L, n)
    if name == "frag":
        # n 64-KiB payloads as the reference sends them (SURVEY.md 8(a) note): each is
        # fragmented into 49 datagrams at the default MTU, 48 of 1392 B (fragment payload
        # MTU - 32 = 1360 B plus 32 B of headers, src/c/peer.rs:181-192) and one of
        # 256 + 32 = 288 B, one checksum per datagram; packed back to back.
        lengths = np.tile(np.array([1392] * 48 + [288], dtype=np.uint32), n)
    else:
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
    out = torch.empty(lengths.size, dtype=torch.int32, device=dev)
    step = lambda: rea.crc32_batch(data, offsets=off, lengths=ln, out=out)  # noqa: E731
    return step, total, lengths.size, out, ("ragged", data, offsets, lengths)


def verify_sample(out, spec, limit=20000) -> None:
    """Bit-exact check of a sample of this rank's outputs against the oracle (not timed)."""
    import _oracle
    from _data import packed_offsets

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


# --------------------------------------------------------------------------------------
# CPU baseline
# --------------------------------------------------------------------------------------

def host_cpus() -> dict:
    """What this process may run on: `nproc` (the affinity mask), the cgroup CPU quota,
    the machine's CPU count and the CPU model."""
    model = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    try:
        nproc = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        nproc = os.cpu_count() or 1
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, period = f.read().split()[:2]
            if q != "max":
                quota = float(q) / float(period)
    except (OSError, ValueError):
        pass
    threads = nproc if quota is None else max(1, min(nproc, int(math.ceil(quota))))
    threads = min(threads, 256)  # the oracle's thread limit (oracle/crc32_oracle.c)
    return {"model": model, "nproc": nproc, "cgroup_cpus": quota, "machine_cpus": os.cpu_count(),
            "threads": threads}


def cpu_baseline(seconds: float = 10.0) -> dict:
    """src/crc32.rs restated in C (oracle/), timed on this host: BASELINE configs[0]."""
    import _oracle
    from _data import ENET_SEED, splitmix64_bytes

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
    cpus = host_cpus()
    threads = cpus["threads"]
    reps = max(8, 2 * threads)  # every thread gets >= 2 x 4096 packets
    big = np.tile(data, reps)
    mt_times = []
    t_end = time.perf_counter() + seconds / 2
    while time.perf_counter() < t_end or len(mt_times) < 10:
        t0 = time.perf_counter()
        _oracle.crc32_uniform(big, L, L, reps * n, threads=threads)
        mt_times.append(time.perf_counter() - t0)
    multi = reps * n * L / float(np.median(mt_times)) / 2**30
    return {"value": round(single, 4), "unit": "GiB/s", "cores": 1, "kind": "port",
            "sample": f"4096 x 1200 B (BASELINE configs[0]), one crc32 call per packet, median of "
                      f"{len(times)} passes over ~{seconds:.0f} s; C restatement of src/crc32.rs (no rustc here)",
            "cpu_model": cpus["model"],
            "all_cores": {"value": round(multi, 4), "unit": "GiB/s", "cores": threads,
                          "sample": f"{reps} x 4096 x 1200 B split over {threads} threads "
                                    f"(nproc {cpus['nproc']}, cgroup quota {cpus['cgroup_cpus']}, "
                                    f"machine CPUs {cpus['machine_cpus']}), median of {len(mt_times)} passes"}}


def range_cpu_baseline(spec, seconds: float = 5.0) -> dict:
    """src/c/compress.rs restated in C (oracle/range_coder_oracle.c) on one host core."""
    import _range_oracle as ro
    from _data import packed_offsets

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
            "cpu_model": host_cpus()["model"],
            "sample": f"first 4096 packets of the workload ({nb} B), one compress call per packet, median of "
                      f"{len(times)} passes; C restatement of src/c/compress.rs (no rustc here)"}


# --------------------------------------------------------------------------------------
# secondary measurements (N = 1 only)
# --------------------------------------------------------------------------------------

def range_decompress_rate(spec, res, steps: int = 3) -> dict:
    """Decompress the step's coded packets back (device-resident), timed on the current stream."""
    import torch

    import rusty_enet_amd as rea

    _, host, offsets, lengths, data, off, ln = spec
    c_out, c_off, c_sizes = res["out"]
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
            "compressed_fraction": round(float(c_sizes.to(torch.int64).sum().item()) /
                                         float(ln.to(torch.int64).sum().item()), 4)}


def end_to_end(dev, n: int = 1 << 18, L: int = 1200) -> dict:
    """Host buffers -> pinned staging -> H2D -> kernel -> D2H (enet_crc32_ragged_host),
    plus the per-call latency of the drop-in hook (enet_crc32_iov, one datagram)."""
    import _oracle
    from _data import ENET_SEED, splitmix64_bytes

    import rusty_enet_amd as rea

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
    if ctx.crc32(pkt) != _oracle.crc32(pkt):
        raise SystemExit("bench: per-call checksum differs from the oracle")
    from rusty_enet_amd import _native

    variants = {}
    for name, mode in (("copy", _native.ENET_CRC_PERCALL_COPY), ("zerocopy", _native.ENET_CRC_PERCALL_ZEROCOPY),
                       ("persistent", _native.ENET_CRC_PERCALL_PERSISTENT)):
        ctx.set_percall_mode(mode)
        if ctx.crc32(pkt) != _oracle.crc32(pkt):
            raise SystemExit(f"bench: per-call ({name}) checksum differs from the oracle")
        for _ in range(50):
            ctx.crc32(pkt)
        calls = 2000
        t0 = time.perf_counter()
        for _ in range(calls):
            ctx.crc32(pkt)
        variants[name] = round((time.perf_counter() - t0) / calls * 1e6, 2)
    ctx.set_percall_mode(_native.ENET_CRC_PERCALL_ZEROCOPY)  # stops the server wave
    per_call_us = variants["zerocopy"]  # the context's default mode (ENET_CRC_PERCALL_ZEROCOPY, ABI >= 5)
    # Floor of any per-call GPU path: one trivial kernel launch + stream synchronize.
    import torch

    x = torch.zeros(1, device=dev)
    for _ in range(50):
        x.add_(1)
        torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(2000):
        x.add_(1)
        torch.cuda.synchronize()
    floor_us = (time.perf_counter() - t0) / 2000 * 1e6
    # The reference's own per-call cost for the same datagram: the oracle's Sarwate loop on one core.
    t0 = time.perf_counter()
    for _ in range(2000):
        _oracle.crc32(pkt)
    cpu_call_us = (time.perf_counter() - t0) / 2000 * 1e6
    ctx.close()
    return {"value": round(rate, 3), "unit": "GiB/s", "path": "enet_crc32_ragged_host",
            "sample": f"{n} x {L} B from pageable host memory, median of 5 passes",
            "per_call_us": round(per_call_us, 2),
            "per_call_variants_us": variants,
            "per_call_cpu_oracle_us": round(cpu_call_us, 2),
            "per_call_floor_us": round(floor_us, 2),
            "per_call_sample": "enet_crc32_iov on one 1392-B datagram (the HostSettings::checksum hook), mean of 2000, "
                               "default mode (zero-copy launch; variants: copy, zero-copy launch, opt-in persistent "
                               "server wave); "
                               "cpu: the C restatement of src/crc32.rs on the same datagram through ctypes; floor: one "
                               "trivial torch kernel launch + torch.cuda.synchronize",
            "ring": ring_rate(dev, L)}


def ring_rate(dev, L: int = 1200, nslots: int = 4, per_slot: int = 40000, rounds: int = 8) -> dict:
    """Pinned receive ring (enet_crc_ring_*): packets already in pinned slot memory,
    H2D + kernel + D2H of each slot on its own stream, slots overlapped."""
    import _oracle
    from _data import ENET_SEED, splitmix64_bytes

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


VERIFY_BATCHES = (16, 32, 64, 128, 256, 512, 1024, 4096, 16384)


def verify_batch(dev, batch: int = 256, reps: int = 200) -> dict:
    """The receive path at the reference's own batch size: enet_protocol_receive_incoming_commands
    takes at most 256 datagrams per service() (src/c/protocol.rs:1655) and checksums each one
    as it handles it (:1470-1502).  Per-batch microseconds for B ragged datagrams of U{64..1392}
    B from host memory: enet_crc32_ragged_host (pageable, staged through pinned memory) plus
    the per-datagram slot correction (enet_crc32_slot_adjust, as the receive loop would call it);
    one pinned ring slot (submit + wait); the whole Python mirror protocol.verify_received; and
    the reference's cost, B calls of the C restatement of src/crc32.rs on one core.  Each GPU
    path is checked bit-exact against the oracle first; the crossover is the smallest batch
    in VERIFY_BATCHES at which the host path beats the one-core CPU."""
    import ctypes

    import _oracle
    from _data import ENET_SEED, packed_offsets, ragged_lengths, splitmix64_bytes

    import rusty_enet_amd as rea
    from rusty_enet_amd import _native, protocol
    from rusty_enet_amd.ring import ReceiveRing

    def med(fn, k):
        fn()
        ts = []
        for _ in range(k):
            t0 = time.perf_counter()
            fn()
            ts.append(time.perf_counter() - t0)
        return float(np.median(ts)) * 1e6

    def sample(b, seed):
        ln = ragged_lengths(ENET_SEED + seed, b, lo=64, hi=1392)
        off = packed_offsets(ln)
        return splitmix64_bytes(ENET_SEED + seed + 1, int(ln.sum())), off, ln

    lib = _native.lib()
    adj = lib.enet_crc32_slot_adjust
    ctx = rea.Context(dev.index or 0)
    rows = {}
    for b in sorted(set(VERIFY_BATCHES) | {batch}):
        data, off, ln = sample(b, 300 + b)
        want = _oracle.crc32_ragged(data, off, ln)
        if not np.array_equal(ctx.crc32_ragged_host(data, off, ln), want):
            raise SystemExit(f"bench: {b}-datagram host batch differs from the oracle")
        out = np.empty(b, dtype=np.uint32)
        args = (ctx.handle, data.ctypes.data, off.ctypes.data, ln.ctypes.data, b, out.ctypes.data)
        host_us = med(lambda: lib.enet_crc32_ragged_host(*args), reps)
        cpu_us = med(lambda: _oracle.crc32_ragged(data, off, ln), reps)  # one C loop over B datagrams
        rows[b] = {"host_us": round(host_us, 1), "cpu_1core_us": round(cpu_us, 1),
                   "bytes": int(ln.sum())}
    data, off, ln = sample(batch, 300 + batch)
    crcs = ctx.crc32_ragged_host(data, off, ln)
    # the receive loop's slot correction (connect_id instead of the wire value), one C call per
    # datagram; the same loop with bytes_after_slot = 0 (no table steps) is the ctypes cost
    real_args = [(int(c), 0x11223344, 0x55667788, int(n) - 6) for c, n in zip(crcs, ln)]
    zero_args = [(int(c), 0x11223344, 0x55667788, 0) for c in crcs]
    slot_us = med(lambda: [adj(*a) for a in real_args], 50)
    call_us = med(lambda: [adj(*a) for a in zero_args], 50)
    with ReceiveRing(dev.index or 0, nslots=1, slot_bytes=batch * 1392, slot_packets=batch) as ring:
        r_data, r_off, r_ln, r_crc = ring.slot(0)
        r_data[:data.size] = data
        r_off[:batch] = off
        r_ln[:batch] = ln
        ring.submit(0, batch)
        ring.wait(0)
        if not np.array_equal(r_crc[:batch], crcs):
            raise SystemExit("bench: ring slot checksums differ")
        ring_us = med(lambda: (ring.submit(0, batch), ring.wait(0)), reps)
    dgrams = [bytes(data[int(o):int(o) + int(n)]) for o, n in zip(off, ln)]
    # datagrams as a client with peer id 7 sends them: the slot holds the checksum with the
    # connect_id in it, so every one is accepted
    conn = 0x0BADF00D
    dg = []
    for d in dgrams:
        a = bytearray(d)
        a[0], a[1] = 0x00, 0x07  # peer id 7, no flags: header 2 + 4
        dg.append(a)
    protocol.insert_outgoing(dg, [2] * batch, [conn] * batch, ctx=ctx)
    ok = protocol.verify_received(dg, lambda pid: conn, ctx=ctx)
    if not all(ok):
        raise SystemExit("bench: verify_received rejected a valid datagram")
    proto_us = med(lambda: protocol.verify_received(dg, lambda pid: conn, ctx=ctx), 50)
    ctx.close()
    cross = next((b for b in sorted(rows) if rows[b]["host_us"] < rows[b]["cpu_1core_us"]), None)
    r = rows[batch]
    return {"batch": batch, "unit": "us per batch",
            "host_us": r["host_us"], "slot_adjust_us": round(max(slot_us - call_us, 0.0), 1),
            "ring_us": round(ring_us, 1), "cpu_1core_us": r["cpu_1core_us"],
            "protocol_verify_received_us": round(proto_us, 1), "bytes": r["bytes"],
            "crossover_batch": cross,
            "sweep": {str(b): rows[b] for b in sorted(rows)},
            "sample": f"{batch} datagrams of U{{64..1392}} B (the reference's receive batch, src/c/protocol.rs:1655), "
                      f"median of {reps}; host: enet_crc32_ragged_host from pageable memory; slot_adjust: "
                      f"{batch} enet_crc32_slot_adjust calls less the same calls with 0 bytes after the slot "
                      "(the ctypes cost); ring: one pinned ring slot "
                      "submit + wait; protocol: the Python mirror verify_received (header parse, one GPU pass, "
                      "per-datagram correction); cpu: the C restatement of src/crc32.rs over the same datagrams on "
                      "one core; crossover: smallest batch of the sweep where host_us < cpu_1core_us"}


# --------------------------------------------------------------------------------------
# roofline evidence
# --------------------------------------------------------------------------------------

CEILING_LIB = os.path.join(REPO, "tools", "lib", "libenet_read_ceiling.so")
CEILING_PRE_LAUNCHES = 40  # per read-ceiling variant before the main line's warmup (~30 ms of load)


class ReadCeiling:
    """tools/ceiling/read_ceiling.hip: a pure streaming read (16-B loads, XOR only) of the
    same device buffer the bench checksums, launched on torch's current stream.  Its best
    variant's rate is the same-process ceiling the kernel is stated against
    (roofline.read_ceiling_gbs / frac_of_ceiling).  Measurement tooling:
    never on the product path."""

    def __init__(self, dev):
        import ctypes

        import torch

        if not os.path.exists(CEILING_LIB):
            raise FileNotFoundError(f"{CEILING_LIB} not built (make all)")
        self._lib = ctypes.CDLL(CEILING_LIB)
        self._lib.enet_read_ceiling.restype = ctypes.c_int
        self._lib.enet_read_ceiling.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p,
                                                ctypes.c_void_p]
        self._lib.enet_read_ceiling_name.restype = ctypes.c_char_p
        self._lib.enet_read_ceiling_name.argtypes = [ctypes.c_int]
        self._lib.enet_read_ceiling_bytes.restype = ctypes.c_uint64
        self._lib.enet_read_ceiling_bytes.argtypes = [ctypes.c_uint64]
        self.variants = int(self._lib.enet_read_ceiling_variants())
        self.dev = dev
        self._out = torch.zeros(4, dtype=torch.int32, device=dev)

    def name(self, v: int) -> str:
        return self._lib.enet_read_ceiling_name(v).decode()

    def bytes_read(self, nbytes: int) -> int:
        return int(self._lib.enet_read_ceiling_bytes(nbytes))

    def launch(self, v: int, data, nbytes: int) -> None:
        import torch

        stream = torch.cuda.current_stream(self.dev).cuda_stream
        st = self._lib.enet_read_ceiling(v, data.data_ptr(), nbytes, self._out.data_ptr(), stream)
        if st != 0:
            raise RuntimeError(f"enet_read_ceiling({v}): hipError {st}")

    def measure(self, data, nbytes: int, launches: int = 10, variants=None) -> dict:
        """Each variant (default: all): one untimed launch, then `launches` timed back to back
        (HIP events on the launch stream).  Returns the best rate and each variant's."""
        import torch

        stream = torch.cuda.current_stream(self.dev)
        nread = self.bytes_read(nbytes)
        per, index = {}, {}
        for v in (range(self.variants) if variants is None else variants):
            self.launch(v, data, nbytes)
            ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            ev0.record(stream)
            for _ in range(launches):
                self.launch(v, data, nbytes)
            ev1.record(stream)
            torch.cuda.synchronize()
            us = ev0.elapsed_time(ev1) * 1000.0 / launches
            per[self.name(v)] = {"us": round(us, 2), "gbs": round(nread / us / 1e3, 1)}
            index[self.name(v)] = v
        best = max(per, key=lambda k: per[k]["gbs"])
        return {"gbs": per[best]["gbs"], "variant": best, "variant_index": index[best], "bytes": nread,
                "launches": launches, "variants": per}


def open_ceiling(dev):
    """ReadCeiling on `dev`, or None when the tooling library is not built (the line then
    says so instead of failing)."""
    try:
        return ReadCeiling(dev)
    except (OSError, FileNotFoundError):
        return None


def ceiling_fields(ceil, pre: dict | None, data, nbytes: int, achieved_gbs: float) -> dict:
    """The same-buffer read ceiling around a timed region: `pre` was measured (all variants)
    just before the warmup steps, this measures the best variant again right after the timed
    steps; frac_of_ceiling = the kernel's algorithmic GB/s / that rate."""
    if ceil is None or pre is None:
        return {"read_ceiling_gbs": None, "frac_of_ceiling": None,
                "read_ceiling": {"note": f"{CEILING_LIB} not built"}}
    post = ceil.measure(data, nbytes, launches=20, variants=[pre["variant_index"]])
    return {"read_ceiling_gbs": post["gbs"], "frac_of_ceiling": round(achieved_gbs / post["gbs"], 4),
            "read_ceiling": {"after_gbs": post["gbs"], "before_gbs": pre["gbs"], "variant": pre["variant"],
                             "bytes": post["bytes"], "before_variants": pre["variants"],
                             "what": "tools/ceiling/read_ceiling.hip: the same device buffer read once with 16-B "
                                     "loads and an XOR, best of its variants measured before the warmup steps "
                                     f"({CEILING_PRE_LAUNCHES} launches each, ~30 ms of load, which also takes "
                                     "the GPU through its clock transient, DESIGN.md §5) and that variant "
                                     "again right after the timed steps "
                                     "(after_gbs = read_ceiling_gbs, 20 launches)"}}


def kernel_source_hash() -> str:
    h = hashlib.sha256()
    for name in KERNEL_SOURCES:
        path = os.path.join(REPO, "rusty_enet_amd", "csrc", name)
        if os.path.exists(path):
            with open(path, "rb") as f:
                h.update(name.encode() + b"\0" + f.read())
    return h.hexdigest()[:16]


def load_pmc_traffic(config: str):
    """HBM bytes per launch of the dominant kernel from profiles/pmc_traffic.json, but only
    when it was measured on the kernel sources as they are now (else None)."""
    path = os.path.join(REPO, "profiles", "pmc_traffic.json")
    try:
        with open(path) as f:
            v = json.load(f).get(config)
    except (OSError, ValueError):
        return None, None
    if not v or v.get("source_hash") != kernel_source_hash():
        return None, None
    return v.get("hbm_bytes_per_launch"), v.get("source")


def range_roofline(nbytes: int, kernel_ms: float, kernel_ms_max: float) -> dict:
    """The range coder is bound by dependent arena accesses (each 16-B node
    read-modify-write is its own memory transaction), not by streaming bandwidth.  With
    the HBM read + write requests per launch from the committed profile (TCC_EA0_RDREQ,
    TCC_EA0_WRREQ; same kernel sources), the achieved rate is expressed as 64-B requests
    per second against the HBM's 8 TB/s / 64 B = 125 G requests/s; without it, only the
    input rate is reported."""
    achieved_in = nbytes / (kernel_ms / 1000.0) / 1e9
    path = os.path.join(REPO, "profiles", "pmc_traffic.json")
    req = None
    try:
        with open(path) as f:
            v = json.load(f).get("range")
        if v and v.get("source_hash") == kernel_source_hash():
            req = v.get("read_requests_per_launch")
            if req and v.get("write_requests_per_launch"):
                req += v["write_requests_per_launch"]
    except (OSError, ValueError):
        pass
    out = {"bound": "latency", "input_gbs": round(achieved_in, 3), "kernel_ms": round(kernel_ms, 3),
           "kernel_ms_max_rank": round(kernel_ms_max, 3),
           "note": "dependent 16-B arena node accesses per input byte; see DESIGN.md §11"}
    if req:
        rate = req / (kernel_ms / 1000.0) / 1e9
        out.update({"achieved": round(rate, 2), "peak": 125.0, "unit": "G read requests/s",
                    "frac": round(rate / 125.0, 4), "traffic": req * 64})
    else:
        out.update({"achieved": None, "peak": 125.0, "unit": "G read requests/s", "frac": None, "traffic": None})
    return out


def time_steps(step, steps: int, barrier, dev) -> tuple[float, float]:
    """(wall seconds, mean ms per launch on the launch stream) over exactly `steps` steps."""
    import torch

    stream = torch.cuda.current_stream(dev)  # the stream crc32_batch launches on
    ev0 = torch.cuda.Event(enable_timing=True)
    ev1 = torch.cuda.Event(enable_timing=True)
    barrier()
    t0 = time.perf_counter()
    ev0.record(stream)
    for _ in range(steps):
        step()
    ev1.record(stream)
    barrier()
    wall = time.perf_counter() - t0
    return wall, ev0.elapsed_time(ev1) / steps


def shard_2m(dev, rank: int, steps: int, warmup: int, barrier) -> dict:
    """The N > 1 per-GPU shard (2M x 1200 B) timed on this GPU, at N = 1."""
    return uniform_point(dev, rank, CONFIGS["uniform"][2], 1200, steps, warmup, barrier)


def uniform_point(dev, rank: int, n: int, L: int, steps: int, warmup: int, barrier) -> dict:
    """n x L-byte uniform packets timed on this GPU (verified on a sample first)."""
    return config_point("uniform", dev, rank, n, steps, warmup, barrier, length=L)


def device_record(dev, rank: int) -> dict:
    """Which physical GPU this rank ran on (gathered into the line's `devices` field)."""
    import torch

    p = torch.cuda.get_device_properties(dev)
    return {"rank": rank, "device": dev.index, "name": p.name,
            "pci": f"{p.pci_domain_id:04x}:{p.pci_bus_id:02x}:{p.pci_device_id:02x}", "uuid": str(p.uuid)}


def gather_objects(obj, world: int) -> list:
    """obj from every rank (gloo), rank order; [obj] without a process group."""
    if world == 1:
        return [obj]
    import torch.distributed as dist

    out = [None] * world
    dist.all_gather_object(out, obj)
    return out


def all_ranks_point(name: str, dev, rank: int, world: int, n: int, steps: int, warmup: int, barrier) -> dict:
    """config_point on every rank (each on its own GPU, same per-GPU shard), reduced like the
    main line: max over ranks of the wall and kernel times; `value` is the aggregate over
    all ranks (world x per-GPU bytes / the slowest rank's time)."""
    from rusty_enet_amd.shards import max_over_ranks

    r = config_point(name, dev, rank, n, steps, warmup, barrier)
    ms, kms = max_over_ranks([r["ms_per_step"], r["kernel_ms"]])
    out = dict(r)
    out.update({"n_gpus": world, "ms_per_step": round(ms, 5), "kernel_ms": round(kms, 5),
                "value": round(world * r["bytes"] / (ms / 1000.0) / 2**30, 2),
                "frac": round(r["bytes"] / (kms / 1000.0) / 1e9 / HBM_PEAK_GBS, 4),
                "note": "value: all ranks' bytes / the slowest rank's time; frac: per GPU, slowest rank"})
    return out


SUSTAIN_MS = 60.0  # extra points: timed after at least this much of their own load (config_point)


def config_point(name: str, dev, rank: int, n: int, steps: int, warmup: int, barrier,
                 length: int | None = None) -> dict:
    """One more workload timed on this GPU after the main line (verified on a sample first):
    the N = 1 line carries the other BASELINE configs' per-GPU shapes next to G1.  Timed twice:
    `cold` right after the line's warmup, and the point's own numbers once the workload has
    run for SUSTAIN_MS (the sustained rate a receive path under load sees)."""
    import torch

    step, nbytes, npk, out, spec = make_workload(name, rank, n, dev, length=length)
    step()
    torch.cuda.synchronize()
    verify_sample(out, spec)
    ceil = open_ceiling(dev)
    pre = ceil.measure(spec[1], nbytes) if ceil else None
    for _ in range(warmup):
        step()
    wall_c, kms_c = time_steps(step, steps, barrier, dev)  # right after the line's own warmup
    # Sustained: the ragged kernel's launches speed up over its first ~30 ms of load (power
    # management; profiles/r04/rramp/ragged_series.txt, 193 -> 150 us), so every point is
    # timed again after at least SUSTAIN_MS of this workload's launches.
    extra = max(0, math.ceil(SUSTAIN_MS / max(kms_c, 1e-3)) - warmup - steps)
    for _ in range(extra):
        step()
    wall, kms = time_steps(step, steps, barrier, dev)
    ms = wall * 1000.0 / steps
    res = {"packets": npk, "bytes": nbytes, "ms_per_step": round(ms, 5),
           "value": round(nbytes / (ms / 1000.0) / 2**30, 2), "unit": "GiB/s",
           "kernel_ms": round(kms, 5), "frac": round(nbytes / (kms / 1000.0) / 1e9 / HBM_PEAK_GBS, 4),
           "timed_after_launches": warmup + steps + extra,
           "cold": {"kernel_ms": round(kms_c, 5), "frac": round(nbytes / (kms_c / 1000.0) / 1e9 / HBM_PEAK_GBS, 4),
                    "ms_per_step": round(wall_c * 1000.0 / steps, 5), "timed_after_launches": warmup}}
    cf = ceiling_fields(ceil, pre, spec[1] if ceil else None, nbytes, nbytes / (kms / 1000.0) / 1e9)
    res["read_ceiling_gbs"], res["frac_of_ceiling"] = cf["read_ceiling_gbs"], cf["frac_of_ceiling"]
    if name in ("ragged", "large", "frag") and n == CONFIGS[name][1]:
        res["traffic"] = load_pmc_traffic(name)[0]  # HBM bytes per launch, committed profile, same sources
    del spec, out
    torch.cuda.empty_cache()
    return res


# --------------------------------------------------------------------------------------

def parse_args(argv):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None, help="GPUs (ranks); default WORLD_SIZE or 1")
    ap.add_argument("--steps", type=int, default=None, help="timed steps (default 200; 5 for --config range)")
    ap.add_argument("--warmup", type=int, default=None, help="untimed steps (default 10; 1 for --config range)")
    ap.add_argument("--config", choices=sorted(CONFIGS), default="uniform")
    ap.add_argument("--packets-per-gpu", type=int, default=None,
                    help="override the per-GPU packet count (default: 1M at N = 1, 2M at N > 1 for uniform)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-verify", action="store_true")
    ap.add_argument("--no-e2e", action="store_true", help="skip the end-to-end host-memory measurement")
    ap.add_argument("--no-shard", action="store_true", help="skip the 2M-packet shard measurement at N = 1")
    return ap.parse_args(argv)


def _with_stdout_on_stderr(fn):
    """fn() with file descriptor 1 redirected to descriptor 2 (C-level prints included)."""
    sys.stdout.flush()
    saved = os.dup(1)
    try:
        os.dup2(2, 1)
        return fn()
    finally:
        sys.stdout.flush()
        os.dup2(saved, 1)
        os.close(saved)


def main(argv=None) -> int:
    argv = sys.argv[1:] if argv is None else argv
    args = parse_args(argv)
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and (args.gpus or 1) > 1:
        return spawn(args, argv)
    world = int(env_world or 1)
    if args.gpus is not None and args.gpus != world:
        print(f"bench: --gpus {args.gpus} but WORLD_SIZE={world}", file=sys.stderr, flush=True)
        return 2
    is_range = args.config == "range"
    if args.steps is None:
        args.steps = 5 if is_range else 200
    if args.warmup is None:
        args.warmup = 1 if is_range else 10
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))

    import torch

    if world > 1:
        import torch.distributed as dist

        # Timing reduction only; no data-path collective.  The gloo transport prints its
        # connection messages on stdout (file descriptor 1), where the driver reads rank 0's one
        # JSON line: the init and a first barrier run with descriptor 1 pointed at stderr.
        def _init():
            dist.init_process_group("gloo")
            dist.barrier()

        _with_stdout_on_stderr(_init)
    shared = os.environ.get("BENCH_SHARE_GPUS") == "1" and torch.cuda.device_count() < world
    dev = torch.device("cuda", local % torch.cuda.device_count() if shared else local)
    torch.cuda.set_device(dev)

    def barrier():
        torch.cuda.synchronize()
        if world > 1:
            torch.distributed.barrier()

    npk = packets_per_gpu(args.config, world, args.packets_per_gpu)
    step, nbytes, npk, out, spec = make_workload(args.config, rank, npk, dev)
    step()
    torch.cuda.synchronize()
    if not args.no_verify:
        verify_sample(out, spec)
    # Same-buffer read ceiling, all variants, before the warmup steps (range: not bound by
    # streaming reads, no ceiling).  40 timed launches per variant, ~30 ms of load in all: the
    # shader clock drops within ~5 ms of load after an idle gap and climbs back over ~30 ms
    # (profiles/r05/clock/), so the timed steps of any K start in the sustained
    # state; the line's `cold` block times the same steps inside that window.
    ceil = None if is_range else open_ceiling(dev)
    ceil_pre = ceil.measure(spec[1], nbytes, launches=CEILING_PRE_LAUNCHES) if ceil else None
    for _ in range(args.warmup):
        step()
    wall, kernel_ms = time_steps(step, args.steps, barrier, dev)
    ceil_fields = None if is_range else ceiling_fields(ceil, ceil_pre, spec[1] if ceil else None, nbytes,
                                                      nbytes / (kernel_ms / 1000.0) / 1e9)

    # Cold: the same steps after an idle second, with only 5 launches of
    # warmup and no read-ceiling pass before them: the chip starts high, drops its shader clock
    # after a few ms of load and climbs back over ~30 ms (profiles/r05/clock);
    # a bursty receive path sees this window.  Reported beside the line, never as its value.
    cold = None
    if not is_range and world == 1:
        time.sleep(1.0)
        for _ in range(5):
            step()
        wall_c, kms_c = time_steps(step, min(args.steps, 20), barrier, dev)
        cold = {"kernel_ms": round(kms_c, 5), "frac": round(nbytes / (kms_c / 1000.0) / 1e9 / HBM_PEAK_GBS, 4),
                "steps": min(args.steps, 20), "warmup": 5, "after_idle_s": 1.0}

    from rusty_enet_amd.shards import max_over_ranks

    wall_max, kernel_ms_max = max_over_ranks([wall, kernel_ms])
    ms_per_step = wall_max * 1000.0 / args.steps
    extra = {}
    devices = gather_objects(device_record(dev, rank), world)
    if world > 1 and args.config == "uniform" and not args.packets_per_gpu:
        # BASELINE configs[4] (256K x 64 KiB over 8 GPUs): its per-GPU shard on every rank,
        # in the same process group, after the configs[3] main line.
        del step, out, spec
        torch.cuda.empty_cache()
        extra["large_64k"] = all_ranks_point("large", dev, rank, world, CONFIGS["large"][2], min(args.steps, 50),
                                             args.warmup, barrier)
    if world == 1 and args.config == "uniform" and not args.no_shard and not args.packets_per_gpu:
        del step, out, spec
        torch.cuda.empty_cache()
        extra["shard_2m"] = shard_2m(dev, rank, min(args.steps, 100), args.warmup, barrier)
        # The reference's default MTU (src/consts.rs:32; SURVEY.md 8(a) note): 1M x 1392 B.
        extra["mtu_1392"] = uniform_point(dev, rank, CONFIGS["uniform"][1], 1392, min(args.steps, 100), args.warmup,
                                          barrier)
        # BASELINE configs[2] (G2, ragged) and the per-GPU shard of configs[4] (G4, 32,768 x
        # 64 KiB): the same measurement as `--config ragged` / `--config large`.
        extra["ragged_g2"] = config_point("ragged", dev, rank, CONFIGS["ragged"][1], min(args.steps, 100),
                                          args.warmup, barrier)
        extra["large_64k"] = config_point("large", dev, rank, CONFIGS["large"][1], min(args.steps, 50),
                                          args.warmup, barrier)
        # The same 32,768 x 64 KiB payloads as the reference checksums them: 49 datagrams each.
        extra["frag_64k"] = config_point("frag", dev, rank, CONFIGS["large"][1], min(args.steps, 50),
                                         args.warmup, barrier)

    if rank == 0:
        total_bytes = nbytes * world
        value = total_bytes / (ms_per_step / 1000.0) / 2**30
        achieved = nbytes / (kernel_ms / 1000.0) / 1e9  # per-GPU algorithmic GB/s (rank 0)
        traffic, traffic_src = load_pmc_traffic(args.config)
        line = {
            "metric": RANGE_METRIC if is_range else METRIC, "value": round(value, 2), "unit": "GiB/s",
            "n_gpus": world, "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms_per_step, 5),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u8",
            "data": "synthetic (torch.randint bytes on device, seeded)",
            "config": {"workload": f"{npk} x " + CONFIGS[args.config][0] + " per GPU", "packets_per_gpu": npk,
                       "bytes_per_gpu": nbytes, "parallelism": f"{world} independent shards, no collective"
                       + (" (REHEARSAL: ranks share GPUs)" if shared else "")},
            "hbm_frac": round(achieved / HBM_PEAK_GBS, 4),
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                         "traffic_source": traffic_src, "kernel_source_hash": kernel_source_hash(),
                         "kernel_ms": round(kernel_ms, 5), "kernel_ms_max_rank": round(kernel_ms_max, 5)},
        }
        if ceil_fields:
            line["roofline"].update(ceil_fields)
        if cold:
            line["roofline"]["cold"] = cold
        line.update(extra)
        line["devices"] = devices
        if is_range:
            line["data"] = "synthetic compressible ENet-like bytes (tests/_data.enet_like_bytes, seeded)"
            line["config"]["workers"] = RANGE_WORKERS
            line["roofline"] = range_roofline(nbytes, kernel_ms, kernel_ms_max)
            if world == 1:
                line["decompress"] = range_decompress_rate(spec, out)
        if world == 1 and args.cpu_seconds > 0:
            line["cpu_baseline"] = range_cpu_baseline(spec) if is_range else cpu_baseline(args.cpu_seconds)
        if world == 1 and not args.no_e2e and not is_range:
            line["end_to_end"] = end_to_end(dev)
            line["verify_256"] = verify_batch(dev)
        print(json.dumps(line), flush=True)
    if world > 1:
        torch.distributed.barrier()
        torch.distributed.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
