"""Host model of the ragged kernels' addressing (rusty_enet_amd/csrc/crc32_kernels.hip): the
product's crc32_ragged_jobs_kernel (8 lanes x 128-B pieces per packet, 8 packets per round,
ring of 3), and the round-4 measurement builds crc32_ragged16_kernel (4 lanes x 64-B pieces,
16 packets per round) and crc32_ragged16w_kernel (16 packets loaded as 8 lanes x 128-B
pieces, two DMA instructions per slot, ring of 2), parked in
profiles/r04/parked/round4_measurement_builds.patch.  Job partition, per-packet records (ragged_record4 / ragged_record), the
class sort and round headers of the job build, each DMA lane's round plan
(round16_from_record / dma_plan_w) and the source of every LDS-DMA the round bodies issue.
No GPU.

Invariants checked on the GPU tests' batch shapes:
  * no DMA source outside the caller's buffer (below base & ~3, or past the last 4-byte word);
  * a lane reads real bytes exactly at the slots whose chunk overlaps its packet (the zero
    chunk before), so the Horner streams see the packet and nothing else;
  * in the unrolled (fast) bodies, every lane's top slot lies in the first ring-length slots
    (the ones the previous round issued with per-lane sources) and in [B, B + spread], and
    every later slot -- read without a per-lane check -- is inside its packet.
Test infrastructure only; mirrors the kernel statement by statement where it matters."""
import zlib

import numpy as np
import pytest

from _data import ENET_SEED, packed_offsets, ragged_lengths

from dataclasses import dataclass


@dataclass(frozen=True)
class Kernel:
    lanes: int        # DMA lanes per packet (16-B chunk k of a piece)
    ring: int         # ring slots per wave
    job_packets: int  # packets per job at most
    min_rounds: int   # fewest rounds per job launch_ragged may choose
    class_long: int   # step counts >= this (or near the base) take the generic body
    max_spread: int   # fast rounds: max - min step count at most
    packets: int = 16  # per round

    @property
    def step(self):
        return 16 * self.lanes

    @property
    def fast_max(self):
        return self.class_long - 1


R16 = Kernel(lanes=4, ring=3, job_packets=512, min_rounds=16, class_long=24, max_spread=2)
R16W = Kernel(lanes=8, ring=2, job_packets=256, min_rounds=16, class_long=14, max_spread=1)
# crc32_ragged_jobs_kernel (the product): 8 packets per round, top slots B .. B + 1
# (any in ring-length rounds).  The model sends near-base packets to the generic body (the
# kernel only the rounds with an actual fallback lane): it checks a subset of the fast rounds.
R8 = Kernel(lanes=8, ring=3, job_packets=256, min_rounds=16, class_long=15, max_spread=1, packets=8)
KERNELS = {"r16": R16, "r16w": R16W, "r8": R8}
SORT_MIN = 4096


def job_shape(K: Kernel, count: int, cus: int = 256):
    best = None
    max_rounds = K.job_packets // K.packets
    for rj in range(max_rounds, K.min_rounds - 1, -1):
        p = rj * K.packets
        nj = -(-count // p)
        grid = min(nj, cus)
        span = -(-nj // grid) * rj
        if best is None or span < best[0]:
            best = (span, p, nj)
    return best[1], best[2]


def record(K: Kernel, sa: int, ln: int, base4: int):
    z = (4 - ((sa + ln) & 3)) & 3 if ln else 0
    a1 = sa + ln + z
    top = sa & ~3
    nwords = (a1 - top) >> 2
    nsteps = -(-nwords // (4 * K.lanes))
    pad = K.step * nsteps - 4 * nwords
    near = top - base4 < 16
    return {"a1": a1, "top": top, "nsteps": nsteps, "pad": pad, "v": sa & 3, "z": z, "near": near}


def check_batch(K: Kernel, offsets, lengths, base: int = 0, end: int | None = None):
    count = len(lengths)
    assert count >= SORT_MIN
    base4 = base & ~3
    if end is None:
        end = int(max(int(o) + int(n) for o, n in zip(offsets, lengths)))
    end4 = (end + 3) & ~3  # the kernels read whole 4-byte words
    jp, njobs = job_shape(K, count)
    stats = {"fast": 0, "generic": 0, "dmas": 0}
    for J in range(njobs):
        p0 = J * jp
        n = min(jp, count - p0)
        recs = [record(K, base + int(offsets[p0 + i]), int(lengths[p0 + i]), base4) for i in range(n)]
        cls = [K.class_long if (r["nsteps"] >= K.class_long or r["near"]) else r["nsteps"] for r in recs]
        order = sorted(range(n), key=lambda i: cls[i])  # any order inside a class is what the kernel may produce
        for rj in range(-(-n // K.packets)):
            q0 = rj * K.packets
            members = [order[q] if q < n else None for q in range(q0, q0 + K.packets)]
            valid_n = [recs[i]["nsteps"] for i in members if i is not None]
            nsmin, nsmax = min(valid_n[0], 255), min(valid_n[-1], 255)
            generic = any(cls[i] == K.class_long for i in members if i is not None) or members[-1] is None
            generic = generic or nsmax == 0
            mx = max(valid_n) if generic else nsmax
            ns = max(K.ring, mx)
            B, spread = ns - nsmax, nsmax - nsmin
            fast = (not generic) and ns <= K.fast_max and (ns == K.ring or spread <= K.max_spread)
            stats["fast" if fast else "generic"] += 1
            for g, i in enumerate(members):
                r = recs[i] if i is not None else None
                for k in range(K.lanes):
                    if r is None:
                        a1, nsteps, pad, top = base4, 0, 0, base4
                    else:
                        a1, nsteps, pad, top = r["a1"], r["nsteps"], r["pad"], r["top"]
                    cb = a1 - 16 * (k + 1) - K.step * (ns - 1)
                    top_slot = ns - nsteps
                    rel = K.step - 16 - 16 * k - pad
                    inside = nsteps > 0 and rel > -16
                    fb = False
                    if r is not None and r["near"] and inside and rel < 0:
                        fb = (a1 - (K.step * nsteps - pad)) - base4 < -rel
                    direct = inside and not fb
                    if fast:
                        assert top_slot == ns or (top_slot < K.ring and B <= top_slot <= B + spread), \
                            (J, rj, g, k, top_slot, B, spread, ns)
                    for s in range(ns):
                        chunk = cb + K.step * s
                        needed = r is not None and nsteps > 0 and chunk + 16 > top and chunk < a1
                        if fast and s >= K.ring:  # unconditional source in the unrolled body
                            real = True
                        else:  # ragged_src
                            real = s > top_slot or (s == top_slot and direct)
                        if real:
                            stats["dmas"] += 1
                            assert base4 <= chunk and chunk + 16 <= end4, (J, rj, g, k, s, chunk, base4, end4)
                            assert needed, ("real bytes outside the packet", J, rj, g, k, s)
                        elif needed:
                            # only the fallback lane (its top chunk reaches below the buffer) reads
                            # its words separately; every other needed chunk is read as a DMA
                            assert not fast and s == top_slot and fb, ("needed chunk not read", J, rj, g, k, s)
    return stats


def _shape(name: str):
    rng = np.random.default_rng(zlib.crc32(name.encode()))
    n = 9000
    if name == "g2":
        lengths = ragged_lengths(ENET_SEED, 20_000)
        return packed_offsets(lengths), lengths
    if name == "frag":
        lengths = np.tile(np.array([1392] * 48 + [288], dtype=np.uint32), 200)
        return packed_offsets(lengths) + np.uint64(1), lengths
    if name == "near_base":
        return rng.integers(0, 16, size=n).astype(np.uint64), rng.integers(0, 1500, size=n).astype(np.uint32)
    if name == "every_length":
        lens, offs, pos = [], [], 0
        for ln in range(0, 701):
            for a in range(16):
                pos += a
                offs.append(pos)
                lens.append(ln)
                pos += ln
        return np.array(offs, dtype=np.uint64), np.array(lens, dtype=np.uint32)
    if name == "adjacent_classes":  # sorted rounds straddling two 128-B step classes
        lengths = (rng.integers(2, 11, size=n) * 128 + rng.integers(-20, 21, size=n)).astype(np.uint32)
    elif name == "empties_short":  # zero-length packets among 1-3-step ones
        lengths = np.where(rng.random(n) < 0.3, 0, rng.integers(1, 384, size=n)).astype(np.uint32)
    elif name == "wide_spread":
        lengths = rng.choice(np.array([40, 300, 560, 820, 1080, 1340], dtype=np.uint32), size=n)
    elif name == "tiny":
        lengths = rng.integers(0, 193, size=n).astype(np.uint32)
    elif name == "long_mix":
        lengths = np.where(rng.random(n) < 0.5, rng.integers(1400, 4097, size=n),
                           rng.integers(0, 200, size=n)).astype(np.uint32)
    elif name == "edges":
        lengths = rng.integers(0, 3001, size=5000).astype(np.uint32)
        lengths[rng.integers(0, 5000, size=100)] = 0
    else:  # one_job
        lengths = rng.integers(0, 1500, size=4096 + 17).astype(np.uint32)
    gaps = rng.integers(0, 5, size=lengths.size).astype(np.uint64)
    return (packed_offsets(lengths) + np.cumsum(gaps)).astype(np.uint64) + np.uint64(1), lengths


@pytest.mark.parametrize("kernel", sorted(KERNELS))
@pytest.mark.parametrize("name", ["g2", "frag", "near_base", "every_length", "wide_spread", "tiny", "long_mix",
                                  "edges", "one_job", "adjacent_classes", "empties_short"])
def test_ragged16_addresses(kernel, name):
    offsets, lengths = _shape(name)
    stats = check_batch(KERNELS[kernel], offsets, lengths)
    assert stats["dmas"] > 0
    if name in ("g2", "frag", "every_length", "tiny"):
        assert stats["fast"] > stats["generic"], stats  # the sort leaves nearly all rounds fast
