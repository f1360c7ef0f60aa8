"""Host model of the ragged jobs kernel's line-anchored rounds (round 6, crc32_kernels.hip:
line_round_from_record, line_pair_plan, the kLine fast bodies and line_rotate) against zlib.

A line round holds 8 packets of the same step count n >= 8 (the job sort makes most long
rounds so).  Its compute slots are whole 128-B lines of each packet instead of 128-B pieces
ending at the packet's 4-byte-grid end a1: slot s of packet g is the line NS - 1 - s lines
before the packet's last line, NS = the round's largest line count (n or n + 1) rounded up to
even, so every LDS-DMA instruction reads whole lines (what lets the interior pairs carry the non-temporal hint; tools/lines_probe).

The arithmetic stays the 8-lane Horner of DESIGN.md §3 on the 16-B grid that ends at
E16 = a1 rounded up to 16 (lane k holds the chunks c ≡ k mod 8 counted back from E16):
  * lane k reads chunk (j_last - k) mod 8 of every line, j_last = the E16 chunk's index in
    the last line (the DMA lane puts it at the LDS position lane k reads: rotation j_last + 1);
  * in the last line, the chunks past E16 (lanes k > j_last) and lane 0's words past a1 are
    not multiplied in: those streams keep their value from the slot before ("skip");
  * the r = (E16 - a1) / 4 words between a1 and E16 shift the 4-byte grid against the 16-B
    grid: before the in-lane Horner each lane forms the a1-grid chunk of its class from its
    own words 0 .. 3 - r and lane (k + 1) mod 8's words 4 - r .. 3 (one neighbour exchange per
    round; lane 7 takes lane 0's skipped words, which are one stream step behind);
  * the first line masks the chunks before the packet's first word (zero) and the first word
    (its bytes before sa, plus the initial register) from the same 32-entry mask table.
Then the usual in-lane Horner, the 3-level tree and finish_word(z).  Checked for every lane,
slot and DMA of random rounds (any start phase and length with the same step count, packed or
with gaps, bases anywhere in a line) and the frag_64k shape, against zlib.crc32.
"""
import random
import zlib

import pytest

POLY = 0xEDB88320
T8 = []
for _b in range(256):
    _c = _b
    for _ in range(8):
        _c = (_c >> 1) ^ (POLY if _c & 1 else 0)
    T8.append(_c)


def m8(x):
    return (x >> 8) ^ T8[x & 0xFF]


_OPS = {}


def op_tables(n):
    """M32^n as 4 byte tables: M32^n(x) = XOR_j T[j][byte j of x]."""
    if n not in _OPS:
        tabs = []
        for j in range(4):
            row = []
            for b in range(256):
                x = b << (8 * j)
                for _ in range(4 * n):
                    x = m8(x)
                row.append(x)
            tabs.append(row)
        _OPS[n] = tabs
    return _OPS[n]


def m32n(x, n):
    t = op_tables(n)
    return t[0][x & 0xFF] ^ t[1][(x >> 8) & 0xFF] ^ t[2][(x >> 16) & 0xFF] ^ t[3][x >> 24]


def m8_inv(y):
    # x with m8(x) = y: the table's top byte names the low byte of x
    for b in range(256):
        if (T8[b] >> 24) == (y >> 24):
            return (((y ^ T8[b]) << 8) & 0xFFFFFFFF) | b
    raise AssertionError


def head_k(v):
    x = 0xFFFFFFFF
    for _ in range(v):
        x = m8_inv(x)
    return x


def bswap32(x):
    return int.from_bytes(x.to_bytes(4, "little"), "big")


def finish_word(y, z):
    """M8^(4 - z)(y) = M32(y << 8 z) ^ (y >> (32 - 8 z)) (crc32_kernels.hip: finish_word)."""
    if z == 0:
        return m32n(y, 1)
    return m32n((y << (8 * z)) & 0xFFFFFFFF, 1) ^ (y >> (32 - 8 * z))


def words(b16):
    return [int.from_bytes(b16[4 * i:4 * i + 4], "little") for i in range(4)]


def mask_entry(head, v):
    """fill_top_masks: (m, x) per word for meta head / v; head 5: the whole chunk is zero."""
    m, x = [0xFFFFFFFF] * 4, [0] * 4
    if 1 <= head <= 4:
        j0 = 4 - head
        for i in range(4):
            m[i] = 0 if i < j0 else ((0xFFFFFFFF << (8 * v)) & 0xFFFFFFFF if i == j0 else 0xFFFFFFFF)
            x[i] = head_k(v) if i == j0 else 0
    elif head == 5:
        m = [0] * 4
    return m, x


def record(sa, ln):
    """ragged_record: a1 (end run to the 4-byte grid), z, v, nsteps, pad."""
    z = (4 - (sa + ln) % 4) % 4 if ln else 0
    a1 = sa + ln + z
    top = sa & ~3
    nwords = (a1 - top) >> 2
    nsteps = -(-(-(-nwords // 4)) // 8)
    return dict(a1=a1, z=z, v=sa & 3, top=top, nsteps=nsteps, pad=128 * nsteps - 4 * nwords)


def line_lane(rec, ns, k):
    """line_round_from_record for compute lane k: (top slot, head code, r, skip mask, zmask)."""
    a1, top = rec["a1"], rec["a1"] - (128 * rec["nsteps"] - rec["pad"])
    assert top == rec["top"]
    lines = ((a1 - 1) >> 7) - (top >> 7) + 1
    ts = ns - lines
    j_last = ((a1 - 1) >> 4) & 7
    r = (-a1 >> 2) & 3
    jk = (j_last - k) & 7
    jt, wt = (top >> 4) & 7, (top >> 2) & 3
    head = 5 if jk < jt else (4 - wt if jk == jt else 0)
    skip = 0xF if k > j_last else ((0xF << (4 - r)) & 0xF if k == 0 else 0)
    zm = (0xFFFFFFFF >> (8 * rec["z"])) if k == 0 else 0xFFFFFFFF
    return ts, head, r, skip, zm, lines


def line_dma(rec, ns, lane):
    """line_pair_plan for DMA lane `lane` of its packet: (piece-0 source, first real pair)."""
    a1, top = rec["a1"], rec["top"]
    last_line, first_line = (a1 - 1) & ~127, top & ~127
    lines = (last_line - first_line) // 128 + 1
    h = ((lane >> 3) ^ (lane >> 4)) & 1
    p = lane & 7
    rot = ((a1 - 1) >> 4) + 1
    db = last_line - 128 * (ns - 1 - h) + 16 * ((p + rot) & 7)
    p0 = max(0, (ns - lines - h + 1) >> 1)
    return db, p0, first_line, last_line


def simulate_line_round(mem, pk, debug=None):
    recs = [record(sa, ln) for sa, ln in pk]
    n = recs[0]["nsteps"]
    assert all(r["nsteps"] == n for r in recs) and n >= 8
    ml = max(((r["a1"] - 1) >> 7) - (r["top"] >> 7) + 1 for r in recs)  # the header's n (+ 1)
    assert n <= ml <= n + 1
    ns = (ml + 1) & ~1
    T = ns - ml  # B: tops in T .. T + 1
    # DMA: the LDS image of every pair (2 instructions x 64 lanes x 16 B)
    lds = {}
    for P in range(ns // 2):
        img = bytearray(b"\xee" * 2048)
        for i in range(2):
            for L in range(64):
                g = 4 * i + (L >> 4)
                db, p0, fl, ll = line_dma(recs[g], ns, L)
                src = db + 256 * P
                if P >= p0:
                    assert fl <= src and src + 16 <= ll + 128, ("DMA outside the packet's lines", g, P, L)
                    data = mem[src:src + 16]
                else:
                    data = bytes(16)
                img[1024 * i + 16 * L:1024 * i + 16 * L + 16] = data
        lds[P] = bytes(img)
    crcs = []
    ys = {}
    hs = {}
    for g in range(8):
        for k in range(8):
            lane = 8 * g + k
            ts, head, r, skip, zm, lines = line_lane(recs[g], ns, k)
            assert T <= ts <= T + 1, (ts, T)
            j = g & 3
            rd_a = 1024 * (g >> 2) + 256 * j + 128 * (j & 1) + 16 * (7 - k)
            h = [0, 0, 0, 0]
            for s in range(ns):
                a = rd_a ^ (128 * (s & 1))
                w = words(lds[s >> 1][a:a + 16])
                if s == ts and head:
                    m, x = mask_entry(head, recs[g]["v"])
                    w = [(w[i] & m[i]) ^ x[i] for i in range(4)]
                if s == ns - 1:
                    w = [w[i] & (zm if i + r >= 3 else 0xFFFFFFFF) for i in range(4)]
                new = [m32n(h[i], 32) ^ w[i] for i in range(4)]
                if s == ns - 1:
                    new = [h[i] if (skip >> i) & 1 else new[i] for i in range(4)]
                h = new
            hs[(g, k)] = (h, r)
    for g in range(8):
        for k in range(8):
            h, r = hs[(g, k)]
            nb, _ = hs[(g, (k + 1) & 7)]
            gw = [nb[i - r + 4] if i < r else h[i - r] for i in range(4)]  # line_rotate
            y = gw[0]
            for i in range(1, 4):
                y = m32n(y, 1) ^ gw[i]
            ys[(g, k)] = y
        acc = 0
        for k in range(8):
            acc ^= m32n(ys[(g, k)], 4 * k) if k else ys[(g, k)]
        if debug is not None: debug.append(([ys[(g, kk)] for kk in range(8)], acc))
        reg = finish_word(acc, recs[g]["z"])
        crcs.append(bswap32(~reg & 0xFFFFFFFF))
    return crcs


def check_rounds(seed, trials, layout):
    rng = random.Random(seed)
    for _ in range(trials):
        n = rng.randint(8, 13)
        base = 4096 + rng.randrange(0, 128)
        pk, sa = [], base + rng.randrange(0, 64)
        for g in range(8):
            while True:  # a length with step count n from this start
                ln = rng.randint(128 * (n - 1) - 8, 128 * n + 4)
                if ln > 0 and record(sa, ln)["nsteps"] == n:
                    break
            pk.append((sa, ln))
            sa += ln + (rng.randrange(0, 40) if layout == "gaps" else 0)
        mem = bytes(rng.randrange(256) for _ in range(sa + 512))
        got = simulate_line_round(mem, pk)
        want = [bswap32(zlib.crc32(mem[a:a + ln])) for a, ln in pk]
        assert got == want, (pk, [hex(x) for x in got], [hex(x) for x in want])


def test_line_rounds_packed():
    check_rounds(1, 25, "packed")


def test_line_rounds_with_gaps():
    check_rounds(2, 25, "gaps")


def test_line_rounds_frag_shape():
    """8 consecutive 1392-B datagrams, as frag_64k's rounds, from every 16-B base phase."""
    rng = random.Random(3)
    for ph in range(0, 128, 16):
        base = 4096 + ph
        pk = [(base + 1392 * g, 1392) for g in range(8)]
        mem = bytes(rng.randrange(256) for _ in range(base + 1392 * 8 + 512))
        assert simulate_line_round(mem, pk) == [bswap32(zlib.crc32(mem[a:a + ln])) for a, ln in pk]


@pytest.mark.parametrize("r", [0, 1, 2, 3])
def test_line_rounds_every_grid_offset(r):
    """Every a1 - E16 offset r and every end chunk position j_last, with all start phases."""
    rng = random.Random(10 + r)
    for j_last in range(8):
        for v in range(4):
            n = 9
            pk = []
            sa = 4096 + 4 * rng.randrange(0, 32) + v
            for g in range(8):
                # end so that a1 = E16 - 4 r lands in chunk j_last of its line
                while True:
                    ln = rng.randint(128 * (n - 1) + 1, 128 * n)
                    a1 = record(sa, ln)["a1"]
                    if ((-a1 >> 2) & 3) == r and ((a1 - 1) >> 4) & 7 == j_last and record(sa, ln)["nsteps"] == n:
                        break
                pk.append((sa, ln))
                sa += ln + rng.randrange(0, 9)
            mem = bytes(rng.randrange(256) for _ in range(sa + 512))
            got = simulate_line_round(mem, pk)
            assert got == [bswap32(zlib.crc32(mem[a:a + ln])) for a, ln in pk], (r, j_last, v)
