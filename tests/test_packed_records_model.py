"""Host model of the packed round records (round 6, crc32_kernels.hip: pack_fast / pack_line in
job_build, fast_round_decode / fast_plan_decode / line_round_decode / line_plan_decode in
make_round).

Once a job's round headers are complete the job build writes the records of fast and line
rounds in a form that already holds the round's slot count NS; each lane of a round then
derives its state from it in a few instructions.  The raw decode it replaces
(pair_round_from_record + pair_plan for fast rounds, the round-6 line_round_from_record +
line_pair_plan for line rounds) is restated here from the round-6 sources, and for random
rounds of every shape the job sort makes (G2 lengths, class-sorted, short/empty, partial last
rounds, line rounds of 8..13 steps from any start phase) every lane's top slot, meta fields,
output id, and both DMA packets' pair-0 address and first real pair must be identical.
The decoded plans are the ones tests/test_pairs_model.py and tests/test_line_rounds_model.py
check against the bytes and zlib.
"""
import random

MASK48 = (1 << 48) - 1
MIN_SLOTS, FAST_MAX, LINE_MIN = 4, 14, 8
HEAD_ZERO = 5
META_V, META_EMPTY, META_Z, META_STORE = 3, 1 << 5, 6, 1 << 10
META_R, META_SKIP = 8, 15  # line rounds (packed records moved r from bit 13 to bit 8)


def u32(x):
    return x & 0xFFFFFFFF


def record(sa, ln, lid):
    """ragged_record + the job build's local id: (ax, info)."""
    z = (4 - (sa + ln) % 4) % 4 if ln else 0
    ea = sa + ln + z
    top, a1 = sa & ~3, ea & ~3
    nwords = (a1 - top) >> 2
    nsteps = ((nwords + 3) // 4 + 7) // 8
    pad = 128 * nsteps - 4 * nwords
    ax = a1 | (sa & 3) << 48 | z << 50 | 1 << 53 | lid << 54  # never near the base here
    return ax, nsteps | (pad >> 2) << 26


def fields(ax, info):
    return dict(a1=ax & MASK48, v=(ax >> 48) & 3, z=(ax >> 50) & 3, id=(ax >> 54) & 255,
                nsteps=info & ((1 << 26) - 1), pad=(info >> 26) << 2)


def header(recs, valid, partial):
    """job_build's header word rule: (ns, B, fast, line)."""
    ns_list = [fields(*r)["nsteps"] for r, v in zip(recs, valid) if v]
    mx = max(ns_list) if ns_list else 0
    mn = min(ns_list) if ns_list else 0xFFFFFFFF
    ns = max(MIN_SLOTS, (mx + 1) & ~1)
    B = ns - mx
    two_pairs = ns <= MIN_SLOTS
    lim = ns if two_pairs else B + 1
    fast = mx > 0 and ns <= FAST_MAX and ns - mn <= lim and (not partial or two_pairs)
    extra = False
    for r, v in zip(recs, valid):
        if v:
            f = fields(*r)
            topl = u32(f["a1"] - (128 * f["nsteps"] - f["pad"]))
            lines = ((((u32(f["a1"] - 1)) >> 7) - (topl >> 7)) & 0x1FFFFFF) + 1
            extra |= lines == f["nsteps"] + 1
    ml = mx + (1 if extra else 0)
    nl = (ml + 1) & ~1
    line = (not partial) and mn == mx and LINE_MIN <= mx <= 13 and nl == ns
    if line:
        return nl, nl - ml, True, True
    return ns, B, fast, False


def lane_consts(lane):
    h = ((lane >> 3) ^ (lane >> 4)) & 1
    return lane & 7, 128 * h + 16 * (lane & 7)  # k, dma_off


# ---- raw decodes (before the packed records) ----------------------------------------------------------------
def raw_fast_lane(ax, info, valid, ns, k):
    f = fields(ax, info)
    nsteps = f["nsteps"] if valid else 0
    rel = 112 - 16 * k - f["pad"]
    inside = nsteps > 0 and rel > -16
    head = int(rel / 4) + 4 if inside and rel <= 0 else 0
    meta = head | f["v"] << META_V | (META_EMPTY if nsteps == 0 else 0) | f["z"] << META_Z | (
        META_STORE if valid else 0)
    return ns - nsteps, meta, f["id"]


def raw_fast_plan(ax, info, ns, dma_off):
    f = fields(ax, info)
    piece0 = f["a1"] - 128 * ns
    d = ns - f["nsteps"]
    first = (d >> 1) + ((128 * (d & 1) + f["pad"] + 240 - dma_off) >> 8)
    return (piece0 + dma_off) & ((1 << 64) - 1), first


def raw_line_lane(ax, info, ns, k):
    f = fields(ax, info)
    a1l = u32(f["a1"])
    topl = u32(a1l - (128 * f["nsteps"] - f["pad"]))
    lines = ((((u32(a1l - 1)) >> 7) - (topl >> 7)) & 0x1FFFFFF) + 1
    j_last, r = (u32(a1l - 1) >> 4) & 7, (u32(-a1l) >> 2) & 3
    jk, jt, wt = (j_last - k) & 7, (topl >> 4) & 7, (topl >> 2) & 3
    head = HEAD_ZERO if jk < jt else (4 - wt if jk == jt else 0)
    skip = 0xF if k > j_last else ((0xF0 >> r) & 0xF if k == 0 else 0)
    meta = head | f["v"] << META_V | f["z"] << META_Z | META_STORE | r << META_R | skip << META_SKIP
    return ns - lines, meta, f["id"]


def raw_line_plan(ax, info, ns, lane):
    f = fields(ax, info)
    h, p = ((lane >> 3) ^ (lane >> 4)) & 1, lane & 7
    a1 = f["a1"]
    a1l = u32(a1)
    topl = u32(a1l - (128 * f["nsteps"] - f["pad"]))
    lines = ((((u32(a1l - 1)) >> 7) - (topl >> 7)) & 0x1FFFFFF) + 1
    db = ((a1 - 1) & ~127) - 128 * (ns - 1 - h) + 16 * ((p + (u32(a1l - 1) >> 4) + 1) & 7)
    x = ns - lines - h
    return db, (x + 1) >> 1 if x > 0 else 0


# ---- packed formats ---------------------------------------------------------------
def pack_fast(ax, info, valid, ns):
    f = fields(ax, info)
    nsteps = f["nsteps"] if valid else 0
    pad = f["pad"] if valid else 0
    W = 128 * (ns - nsteps) + pad + 240
    assert W < 4096
    X = ((f["a1"] - 128 * ns) & MASK48) | W << 48
    kt = (127 - pad) >> 4
    ht = 32 - 4 * kt - (pad >> 2) if nsteps else 0
    Y = ht | f["v"] << META_V | (META_EMPTY if nsteps == 0 else 0) | f["z"] << META_Z | (
        META_STORE if valid else 0) | kt << 13 | (ns - nsteps) << 16 | f["id"] << 24
    assert Y < 1 << 32 and ns - nsteps < 16
    return X, Y


def head_table_loop(j_last, jt, ht):
    """Format B's head table by its definition: entry k is the code of chunk (j_last - k) mod 8."""
    tab = 0
    for k in range(8):
        jk = (j_last - k) & 7
        tab |= (HEAD_ZERO if jk < jt else (ht if jk == jt else 0)) << (3 * k)
    return tab


def head_table(j_last, jt, ht):
    """pack_line's closed form: the fields m = 7 - jk, then a 24-bit rotation."""
    rep = HEAD_ZERO * 0x249249
    rev = (rep & u32(0xFFFFFF << (3 * (8 - jt)))) | (ht << (3 * (7 - jt)))
    rot = 3 * (7 - j_last)
    return ((rev >> rot) | u32(rev << (24 - rot))) & 0xFFFFFF


def test_head_table_closed_form():
    for j_last in range(8):
        for jt in range(8):
            for ht in range(1, 5):
                assert head_table(j_last, jt, ht) == head_table_loop(j_last, jt, ht), (j_last, jt, ht)


def pack_line(ax, info, ns):
    f = fields(ax, info)
    a1 = f["a1"]
    a1l = u32(a1)
    topl = u32(a1l - (128 * f["nsteps"] - f["pad"]))
    lines = ((((u32(a1l - 1)) >> 7) - (topl >> 7)) & 0x1FFFFFF) + 1
    j_last, r = (u32(a1l - 1) >> 4) & 7, (u32(-a1l) >> 2) & 3
    jt, ht = (topl >> 4) & 7, 4 - ((topl >> 2) & 3)
    tab = head_table(j_last, jt, ht)
    assert tab == head_table_loop(j_last, jt, ht)
    m = f["v"] | f["z"] << 3 | r << 5
    L = (((a1 - 1) & ~127) - 128 * (ns - 1)) & MASK48
    assert 0 <= ns - lines < 16
    X = L | (j_last | (ns - lines) << 3 | m << 7) << 48
    return X, tab | f["id"] << 24


def fast_lane(Y, k):
    meta = Y if ((Y >> 13) & 7) == k else Y & ~7
    return (Y >> 16) & 15, meta, Y >> 24


def fast_plan(X, dma_off):
    db = (X & MASK48) + dma_off
    return db, (u32((X >> 32) - (dma_off << 16))) >> 24


def line_lane(X, Y, k):
    xh = X >> 32
    j_last, r = (xh >> 16) & 7, (xh >> 28) & 3
    head = (Y >> (3 * k)) & 7
    skip = (0xF if k > j_last else 0) | ((0xF0 >> r) & 0xF if k == 0 else 0)
    meta = head | ((xh >> 20) & 0x3F8) | META_STORE | skip << META_SKIP
    return (xh >> 19) & 15, meta, Y >> 24


def line_plan(X, dma_off):
    h128, p16 = dma_off & 128, (dma_off & 0x70) + 16
    xh = X >> 32
    db = (X & MASK48) + (h128 | ((p16 + 16 * ((xh >> 16) & 7)) & 0x70))
    x = (xh >> 19) & 15
    return db, max(0, (x - (h128 >> 7) + 1) >> 1)


FAST_META_BITS = 0x7FF  # head, v, empty, z, store (the fields a fast body reads)


def check_round(pk, valid, partial):
    recs = [record(sa, ln, 8 * 3 + g) if v else (0, 0) for g, ((sa, ln), v) in enumerate(zip(pk, valid))]
    ns, B, fast, line = header(recs, valid, partial)
    if not (fast or line):
        return None
    # every fast or line header has an unrolled body (the kernel has no fallback for them):
    # pair_round_short (NS 4, B 0..3), pair_round_dispatch (NS 6..14, B 0 / 1), line_round_dispatch
    if line:
        assert (ns, B) in {(8, 0), (10, 0), (12, 0), (14, 0), (10, 1), (12, 1), (14, 1)}, (ns, B)
    else:
        assert (ns == MIN_SLOTS and 0 <= B <= 3) or (ns in (6, 8, 10, 12, 14) and B in (0, 1)), (ns, B)
    for lane in range(64):
        g, (k, dma_off) = lane >> 3, lane_consts(lane)
        ax, info = recs[g]
        dp = [recs[lane >> 4], recs[(lane >> 4) + 4]]
        if line:
            X, Y = pack_line(ax, info, ns)
            assert line_lane(X, Y, k) == raw_line_lane(ax, info, ns, k), (pk, lane)
            for (dax, dinfo) in dp:
                DX, _ = pack_line(dax, dinfo, ns)
                assert line_plan(DX, dma_off) == raw_line_plan(dax, dinfo, ns, lane), (pk, lane)
        else:
            X, Y = pack_fast(ax, info, valid[g], ns)
            ts, meta, ident = fast_lane(Y, k)
            rts, rmeta, rid = raw_fast_lane(ax, info, valid[g], ns, k)
            assert (ts, meta & FAST_META_BITS) == (rts, rmeta & FAST_META_BITS), (pk, valid, lane)
            assert not valid[g] or ident == rid
            for j, (dax, dinfo) in enumerate(dp):
                pv = valid[(lane >> 4) + 4 * j]
                DX, _ = pack_fast(dax, dinfo, pv, ns)
                got_db, got_first = fast_plan(DX, dma_off)
                want_db, want_first = raw_fast_plan(dax, dinfo, ns, dma_off)
                assert got_first == want_first, (pk, valid, lane, j)
                if pv:  # an invalid position's address is never used (its pairs are all checked)
                    assert got_db == want_db, (pk, lane, j)
    return "line" if line else "fast"


def rounds(seed, n, lens_fn, partial_p=0.0):
    rng = random.Random(seed)
    kinds = {"fast": 0, "line": 0, None: 0}
    for _ in range(n):
        lens = lens_fn(rng)
        sa = (1 << 40) + rng.randrange(0, 4096)
        pk = []
        for ln in lens:
            pk.append((sa, ln))
            sa += ln + (rng.randrange(0, 24) if rng.random() < 0.3 else 0)
        valid = [True] * 8
        partial = False
        if rng.random() < partial_p:
            cut = rng.randrange(1, 8)
            valid = [i < cut for i in range(8)]
            partial = True
        kinds[check_round(pk, valid, partial)] += 1
    return kinds


def test_packed_g2_rounds():
    k = rounds(1, 400, lambda r: [r.randint(64, 1392) for _ in range(8)], partial_p=0.1)
    assert k["fast"] > 0


def test_packed_class_sorted_rounds():
    def lens(r):
        c = r.randint(1, 14)
        return [r.randint(max(0, 128 * (c - 1) - 40), 128 * c) for _ in range(8)]
    k = rounds(2, 600, lens, partial_p=0.1)
    assert k["fast"] > 100 and k["line"] > 5


def test_packed_line_rounds_every_step_count():
    """Rounds of 8 equal step counts 8..13 from every start phase: the line rounds."""
    rng = random.Random(3)
    seen = 0
    for n in range(8, 14):
        for ph in range(0, 128, 4):
            for _ in range(3):
                sa = (1 << 40) + ph + rng.randrange(0, 4) * 128
                pk = []
                for _g in range(8):
                    while True:
                        ln = rng.randint(128 * (n - 1) - 8, 128 * n + 4)
                        ax, info = record(sa, ln, 0)
                        if ln > 0 and fields(ax, info)["nsteps"] == n:
                            break
                    pk.append((sa, ln))
                    sa += ln + rng.choice([0, 0, 1, 3, 16])
                seen += check_round(pk, [True] * 8, False) == "line"
    assert seen > 100


def test_packed_short_empty_partial():
    vals = [0, 1, 2, 3, 4, 5, 60, 64, 124, 127, 128, 129, 255, 256, 257, 511, 512]
    k = rounds(4, 600, lambda r: [r.choice(vals) for _ in range(8)], partial_p=0.4)
    assert k["fast"] > 300


def test_empty_rounds_are_not_fast():
    """A round of empty packets only (B = 4) has no fast body: it takes the generic loop."""
    recs = [record((1 << 40) + 8 * g, 0, g) for g in range(8)]
    assert header(recs, [True] * 8, False)[2] is False
    assert check_round([((1 << 40) + 8 * g, 0) for g in range(8)], [True] * 8, False) is None
    assert check_round([((1 << 40) + 8 * g, 0 if g else 5) for g in range(8)], [True] * 8, False) == "fast"


def test_frag_shape_rounds():
    """frag_64k: 1392-B datagrams (line rounds) and the 288-B tails (4-slot fast rounds)."""
    for L in (1392, 288):
        for base in range(0, 128, 4):
            sa = (1 << 40) + base
            pk = [(sa + L * g, L) for g in range(8)]
            assert check_round(pk, [True] * 8, False) == ("line" if L == 1392 else "fast")
