"""Host model of the ragged jobs kernel's 256-B pair loads (round 5,
crc32_kernels.hip: PairRing, pair_plan, pair_step).  Restates the kernel's index arithmetic
and checks, for random rounds of 8 packets (empty, invalid, near-base and long packets, odd
and even step counts):

* every DMA source lies inside [base4, a1) of its packet's run, or is the zero chunk;
* what compute lane 8 g + k reads at compute slot s from the LDS pair slot is exactly the
  chunk the round's arithmetic expects there (the 16 bytes ending 16 (k + 8 i) bytes before
  the packet's 4-byte-grid end, i = NS - 1 - s) when that chunk reaches the packet's top
  word and lies in the caller's buffer, zeros otherwise (a top chunk below the buffer is the
  compute lane's own fallback load, not the DMA's);
* each 16-lane quarter of a compute slot's ds_read_b128 covers 256 distinct bytes of one
  256-B bank row (no bank conflicts).
"""
import numpy as np
import pytest

LANES, G, STEP = 64, 8, 128
MIN_SLOTS = 4


def geometry(sa, length):
    """ragged_record: (a1, nsteps, pad) of a packet run to the next 4-byte boundary."""
    z = (4 - (sa + length) % 4) % 4 if length else 0
    ea = sa + length + z
    top, a1 = sa & ~3, ea & ~3
    nwords = (a1 - top) >> 2
    nsteps = ((nwords + 3) // 4 + G - 1) // G
    return a1, nsteps, 128 * nsteps - 4 * nwords, top


def round_slots(nsteps_list):
    """The round header's max step count (valid packets only) -> NS."""
    m = max(nsteps_list)
    return max(MIN_SLOTS, (m + 1) & ~1)


def lane_consts(lane):
    g, k = lane >> 3, lane & 7
    j = g & 3
    rd_a = 1024 * (g >> 2) + 256 * j + 128 * (j & 1) + 16 * (7 - k)
    jd = (lane >> 4) & 3
    h = ((lane >> 3) & 1) ^ (jd & 1)
    dma_off = 128 * h + 16 * (lane & 7)
    return rd_a, dma_off


def simulate_round(mem, base4, packets, valid, rng_dummy=None):
    """packets: list of 8 (sa, length); valid: list of 8 bools.  Returns the LDS image of
    every pair and the per-(lane, slot) data the compute lanes read."""
    geo = [geometry(sa, ln) for sa, ln in packets]
    nsteps = [gg[1] if v else 0 for gg, v in zip(geo, valid)]
    ns = round_slots(nsteps)
    # pair_plan per (lane, DMA packet): an invalid position's record reads as ax = info = 0
    def plan(p, dma_off):
        a1, nst, pad, top = geo[p]
        if not valid[p]:
            a1, nst, pad, near = 0, 0, 0, False
        else:
            near = top - base4 < 16
        piece0 = a1 - STEP * ns
        d = ns - nst
        first = (d >> 1) + ((128 * (d & 1) + pad + 240 - dma_off) >> 8)
        if near:
            x = base4 - piece0 - dma_off
            first = max(first, 0 if x <= 0 else (x + 255) >> 8)
        return piece0 + dma_off, first

    # The round header and the fast rule (make_round): fast rounds issue their own pairs P >= 2
    # unchecked, straight from the plan; every such source must lie inside its packet.
    vs = [n for n, v in zip(nsteps, valid) if v]
    mx, mn = (max(vs), min(vs)) if vs else (0, 0xFFFFFFFF)
    near_round = any(v and geo[p][3] - base4 < 16 for p, v in enumerate(valid))
    B = ns - mx
    lim = MIN_SLOTS if ns == MIN_SLOTS else B + 1
    partial = not all(valid)
    fast = (not near_round) and mx > 0 and ns <= 14 and ns - mn <= lim and (not partial or ns == MIN_SLOTS)
    if fast:
        for P in range(2, ns // 2):
            for i in range(2):
                for L in range(LANES):
                    gp = 4 * i + (L >> 4)
                    dbo, _ = plan(gp, lane_consts(L)[1])
                    src = dbo + 256 * P
                    assert valid[gp] and base4 <= src and src + 16 <= geo[gp][0], ("unchecked", gp, P, L)
    reads = {}
    for P in range(ns // 2):
        lds = np.full(2048, 0xEE, dtype=np.uint8)  # garbage unless written
        for i in range(2):
            for L in range(LANES):
                gp = 4 * i + (L >> 4)
                _, dma_off = lane_consts(L)
                dbo, first = plan(gp, dma_off)
                src = dbo + 256 * P
                real = P >= first
                if real:
                    a1 = geo[gp][0]
                    assert base4 <= src and src + 16 <= a1, (gp, P, L, src, a1)
                    data = mem[src:src + 16]
                else:
                    data = np.zeros(16, dtype=np.uint8)
                lds[1024 * i + 16 * L:1024 * i + 16 * L + 16] = data
        for half in range(2):
            s = 2 * P + half
            addrs = []
            for lane in range(LANES):
                rd_a, _ = lane_consts(lane)
                a = rd_a ^ (128 * half)
                addrs.append(a)
                reads[(lane, s)] = lds[a:a + 16].copy()
            # bank check: each quarter reads 16 distinct 16-B bank groups of a 256-B row
            for q in range(4):
                banks = {(a % 256) // 16 for a in addrs[16 * q:16 * q + 16]}
                assert len(banks) == 16, (P, half, q)
    return ns, geo, reads


def expected(mem, base4, packet, v, ns, lane, s):
    (sa, ln) = packet
    a1, nsteps, pad, top = geometry(sa, ln)
    k = lane & 7
    i = ns - 1 - s
    A = a1 - 16 * (k + 8 * i + 1)
    if not v or A + 16 <= top or A < base4:
        return np.zeros(16, dtype=np.uint8)
    return mem[A:A + 16]


def check(seed, lengths_fn, trials=40):
    rng = np.random.default_rng(seed)
    for _ in range(trials):
        lengths = lengths_fn(rng)
        base = 64 + int(rng.integers(0, 4))  # the caller's buffer starts here
        base4 = base & ~3
        gaps = rng.integers(0, 3, size=8) * (rng.random(8) < 0.3)
        sa, pk = base + int(rng.integers(0, 20)), []
        for ln, gp in zip(lengths, gaps):
            pk.append((sa, int(ln)))
            sa += int(ln) + int(gp)
        mem = rng.integers(0, 256, size=sa + 512, dtype=np.uint8)
        valid = [bool(x) for x in rng.random(8) < 0.95]
        if rng.random() < 0.3:  # the batch's last round: positions past the batch at its end
            cut = int(rng.integers(1, 8))
            valid = valid[:cut] + [False] * (8 - cut)
        ns, geo, reads = simulate_round(mem, base4, pk, valid)
        for lane in range(LANES):
            g = lane >> 3
            for s in range(ns):
                want = expected(mem, base4, pk[g], valid[g], ns, lane, s)
                got = reads[(lane, s)]
                if not np.array_equal(got, want):
                    # the only allowed difference: a fallback top chunk (below the buffer),
                    # which the compute lane loads itself
                    a1, nsteps, pad, top = geo[g]
                    A = a1 - 16 * ((lane & 7) + 8 * (ns - 1 - s) + 1)
                    assert valid[g] and A < base4 < A + 16 and A + 16 > top, (lane, s, A, base4)
                    assert not got.any()


def test_pair_loads_g2_lengths():
    check(1, lambda r: r.integers(64, 1393, size=8))


def test_pair_loads_class_sorted_rounds():
    """Rounds as the job sort makes them: step counts within one or two of each other."""
    def lens(r):
        c = int(r.integers(1, 12))
        return r.integers(max(1, 128 * (c - 1) - 60), 128 * c + 1, size=8)
    check(2, lens)


def test_pair_loads_short_empty_and_long():
    check(3, lambda r: r.choice([0, 1, 2, 3, 5, 60, 64, 127, 128, 129, 511, 1392, 1396, 1791, 1792], size=8))


def test_pair_loads_near_base():
    """Packets starting within 16 B of the buffer base (the fallback top chunk)."""
    check(4, lambda r: r.integers(1, 300, size=8), trials=80)


@pytest.mark.parametrize("ring", [1, 2])
def test_pair_ring_sequence(ring):
    """The pair ring across a wave's rounds (pair_step restated, kPairRing = `ring` pair
    slots): every compute slot reads the (round, pair, half) it consumes from the pair slot
    that pair was loaded into, no pair slot is refilled before its last read, and each
    vmcnt(2 (ring - 1)) wait leaves only the DMAs of pairs issued after the one being read in
    flight (DMAs complete in issue order).  A job build's descriptor DMAs (3 per build) go out
    at random round starts; its own wait, vmcnt(kDescWait = 2) at the end of the round, must
    find them landed.  Pairs 0 and 1 of every round are issued checked: by the round before
    (P < ring) or by the round itself (ring 1: pair 1)."""
    rng = np.random.default_rng(7 + ring)
    for _ in range(200):
        rounds = [2 * int(x) for x in rng.integers(2, 8, size=int(rng.integers(1, 12)))] + [4]  # + a trailing round
        slot_of = {}  # (round, pair) -> LDS pair slot
        dmas = []     # issue order of (round, pair) (2 DMA instructions each)
        reads_left = {}

        checked = {}  # (round, pair) -> issued checked

        def issue(r, P, q, chk):
            assert all(v == 0 for (rr, pp), v in reads_left.items() if slot_of.get((rr, pp)) == q), \
                ("refilled before its last read", r, P, q)
            assert P < rounds[r] // 2
            slot_of[(r, P)] = q
            reads_left[(r, P)] = 2
            checked[(r, P)] = chk
            dmas.extend([("ring", r, P)] * 2)  # two DMA instructions per pair

        def landed(n):  # after vmcnt(n): all but the last n DMA instructions
            return set(dmas[:len(dmas) - n])

        wait = 2 * (ring - 1)
        # prologue: pairs 0 .. ring - 1 of round 0 into pair slots 0 .. ring - 1, then read compute slot 0
        for P in range(ring):
            issue(0, P, P, True)
        assert ("ring", 0, 0) in landed(wait)
        reads_left[(0, 0)] -= 1
        nextv, q = (0, 0, 0), 0
        for r in range(len(rounds) - 1):
            ns = rounds[r]
            job = rng.random() < 0.3
            if job:  # job_dma at the start of the iteration
                dmas.extend([("job", r)] * 3)
            for s in range(ns):
                P, half = s >> 1, s & 1
                assert nextv == (r, P, half), (nextv, r, P, half)
                if half == 0:
                    nxt = (r, P, 1)
                    assert slot_of[(r, P)] == q
                else:
                    nxt = (r + 1, 0, 0) if s == ns - 1 else (r, P + 1, 0)
                    assert slot_of[(nxt[0], nxt[1])] == (q + 1) % ring, (nxt, q)
                    assert ("ring", nxt[0], nxt[1]) in landed(wait), ("not landed", nxt, dmas[-3:])
                reads_left[(nxt[0], nxt[1])] -= 1
                nextv = nxt
                if half == 0:  # pair slot q's last half has been read: refill it with pair P + ring
                    f = P + ring
                    if f < ns // 2:
                        issue(r, f, q, f < 2)  # fast rounds: own pairs unchecked from pair 2 on
                    else:
                        issue(r + 1, f - ns // 2, q, True)
                else:
                    q = (q + 1) % ring
            if job:  # job_build after the round: vmcnt(kDescWait = 2)
                assert ("job", r) in landed(2), ("descriptors not landed", dmas[-6:])
        for (r, P), chk in checked.items():
            assert P >= 2 or chk, ("a round's pair 0 / 1 went out unchecked", r, P)


def test_pair_ring_sequence_staggered():
    """The staggered refill (ENET_CRC_STAGGER, parked in profiles/r05/parked/): the two DMAs of a refill pair go out
    one compute slot apart (instruction 0 after half 0, instruction 1 after half 1, both into the
    pair slot just emptied).  Checked per DMA instruction across a wave's rounds, with the
    descriptor DMAs of a job build (3 per build) issued at random round starts: each compute
    read finds both DMAs of its pair landed after its wait (vmcnt(2) at half 0, vmcnt(1) at
    half 1; DMAs complete in issue order), no pair slot half is refilled before its last read,
    and at every round end the same DMAs are in flight as with whole-pair refills (the next
    round's pair 1), which the job build's own waits count on."""
    rng = np.random.default_rng(11)
    for _ in range(300):
        rounds = [2 * int(x) for x in rng.integers(2, 8, size=int(rng.integers(1, 12)))] + [4]
        dmas = []          # issue order: ("ring", round, pair, instr) or ("job",)
        slot_of = {}       # (round, pair) -> pair slot
        reads_left = {}    # (round, pair) -> reads of that pair still to come (2 halves)

        def issue(r, P, i, q):
            if i == 0:
                assert all(v == 0 for k, v in reads_left.items() if slot_of.get(k) == q), ("refilled early", r, P)
                slot_of[(r, P)] = q
                reads_left[(r, P)] = 2
            else:
                assert slot_of[(r, P)] == q
            dmas.append(("ring", r, P, i))

        def wait(n):  # vmcnt(n): everything but the last n issued has landed
            return set(dmas[:-n] if n else dmas)

        def need(r, P, landed):
            assert ("ring", r, P, 0) in landed and ("ring", r, P, 1) in landed, ("not landed", r, P)

        for i in range(2):
            issue(0, 0, i, 0)
        for i in range(2):
            issue(0, 1, i, 1)
        need(0, 0, wait(2))
        reads_left[(0, 0)] -= 1
        q = 0
        for r in range(len(rounds) - 1):
            ns = rounds[r]
            if rng.random() < 0.3:  # a job build's descriptor DMAs at the round's start
                dmas.extend([("job",)] * 3)
            if r > 0:  # round end invariant: the next round's pair 1 is what is in flight
                ring_tail = [d for d in dmas if d[0] == "ring"][-2:]
                assert ring_tail == [("ring", r, 1, 0), ("ring", r, 1, 1)], ring_tail
            for s in range(ns):
                P, half = s >> 1, s & 1
                f = P + 2
                tgt = (r, f) if f < ns // 2 else (r + 1, f - ns // 2)
                if half == 0:
                    need(r, P, wait(2))           # reading half 1 of pair P
                    reads_left[(r, P)] -= 1
                    issue(tgt[0], tgt[1], 0, q)
                else:
                    nxt = (r + 1, 0) if s == ns - 1 else (r, P + 1)
                    assert slot_of[nxt] == q ^ 1
                    need(nxt[0], nxt[1], wait(1))  # reading half 0 of the next pair
                    reads_left[nxt] -= 1
                    issue(tgt[0], tgt[1], 1, q)
                    q ^= 1
