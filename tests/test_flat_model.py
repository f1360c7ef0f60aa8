"""CPU model of the flat-stream ragged kernels' arithmetic ("Flat-stream
kernels"), checked against zlib's CRC-32 (the same function as src/crc32.rs:39-47).

The GPU kernels compute, per region r of the stream, G_r(x) = the zero-initialised
register of the region's bytes up to x; at each packet boundary x they emit
E(x) = M8^(T - x) G_r(x) (T = the end of the 128-B step holding x), and at each region
end tails[r] = G_r(R1).  The finish pass recovers every packet's checksum by linearity:
    reg = M8^-(T_e - e) [E(e) ^ sum_r M8^(T_e - R1_r) tails[r] ^ M8^(T_e - T_s) E(s)]
          ^ M8^len(0xFFFFFFFF)
This test rebuilds those quantities byte by byte in Python and applies the same formula,
so the algebra the kernels rely on is pinned on the CPU independently of the GPU."""
import random
import zlib

import pytest

POLY = 0xEDB88320
TABLE = []
for b in range(256):
    r = b
    for _ in range(8):
        r = (r >> 1) ^ POLY if r & 1 else r >> 1
    TABLE.append(r)
INV_TOP = {TABLE[b] >> 24: b for b in range(256)}


def reg_of(data: bytes, reg: int) -> int:
    for byte in data:
        reg = (reg >> 8) ^ TABLE[(reg ^ byte) & 0xFF]
    return reg


def m8(reg: int, n: int) -> int:           # n zero bytes: M8^n
    for _ in range(n):
        reg = (reg >> 8) ^ TABLE[reg & 0xFF]
    return reg


def m8_inv(reg: int, n: int) -> int:       # M8^-n (crc32_ops.hpp m8_inverse)
    for _ in range(n):
        b = INV_TOP[reg >> 24]
        reg = (((reg ^ TABLE[b]) << 8) & 0xFFFFFFFF) | b
    return reg


def bswap(x: int) -> int:
    return int.from_bytes(x.to_bytes(4, "little"), "big")


def flat_checksums(buf: bytes, base: int, offsets, lengths, ngroups: int):
    """The kernels' quantities and the finish formula (positions absolute = base + offset)."""
    starts = [base + o for o in offsets]
    ends = [s + n for s, n in zip(starts, lengths)]
    lo = starts[0] & ~127
    hi = max(ends[-1], lo + 1)
    hi = (hi + 127) & ~127
    spg = -(-((hi - lo) // 128) // ngroups)
    rb = spg * 128
    # Stream bytes [a, b).  Below the caller's base the kernels read whatever the memory
    # holds (same page, never part of a packet): junk that cancels in the formula.
    junk = bytes((0xA5 + 7 * i) & 0xFF for i in range(max(0, base - lo)))
    stream = junk + buf
    mem = lambda a, b: stream[a - lo if base > lo else a - base:b - lo if base > lo else b - base]  # noqa: E731

    def region_of(x):       # region with R0 < x <= R1 (x > lo)
        return (x - lo - 1) // rb

    def G(r, x):            # zero-initialised register of region r's bytes [R0, x)
        r0 = lo + r * rb
        return reg_of(mem(r0, x), 0)

    def step_end(x):        # T: end of the step whose (S0, S0 + 128] holds x
        return max((x + 127) & ~127, lo + 128)

    def E(x):
        if x <= lo:
            return 0
        return m8(G(region_of(x), x), step_end(x) - x)

    tails = {}
    out = []
    for s, e, n in zip(starts, ends, lengths):
        if e <= lo:
            out.append(0)
            continue
        te = step_end(e)
        reg = E(e)
        rs = region_of(s) if s > lo else 0
        for r in range(rs, region_of(e)):
            if r not in tails:
                tails[r] = G(r, lo + (r + 1) * rb)
            reg ^= m8(tails[r], te - (lo + (r + 1) * rb))
        if s > lo:
            reg ^= m8(E(s), te - step_end(s))
        reg = m8_inv(reg, te - e) ^ m8(0xFFFFFFFF, n)
        out.append(bswap(~reg & 0xFFFFFFFF))
    return out


def zlib_checksums(buf, offsets, lengths):
    return [bswap(zlib.crc32(buf[o:o + n])) for o, n in zip(offsets, lengths)]


@pytest.mark.parametrize("seed", range(40))
def test_flat_finish_formula_matches_zlib(seed):
    rng = random.Random(seed)
    n = rng.randint(1, 40)
    lengths = [rng.choice([0, 0, 1, 3, 17, 64, 127, 128, 129, 300, rng.randint(0, 700)]) for _ in range(n)]
    gaps = [rng.choice([0, 0, 0, 1, 5, 130, rng.randint(0, 400)]) for _ in range(n)]
    offsets, pos = [], rng.randint(0, 200)
    for ln, gp in zip(lengths, gaps):
        pos += gp
        offsets.append(pos)
        pos += ln
    buf = bytes(rng.getrandbits(8) for _ in range(pos + 64))
    base = rng.choice([0, 5, 64, 1000]) * 128 + rng.randint(0, 127)  # any absolute alignment
    ngroups = rng.choice([1, 2, 3, 7, 16, 64])
    assert flat_checksums(buf, base, offsets, lengths, ngroups) == zlib_checksums(buf, offsets, lengths)


def test_reference_kats_through_the_formula():
    # src/crc32.rs:52 and :54-55 as a two-packet stream (the second is the two slices joined)
    a = bytes([1, 2, 3, 4, 5, 6, 7, 8])
    b = a + bytes([8, 7, 6, 5, 4, 3, 2, 1])
    buf = a + b
    got = flat_checksums(buf, 0, [0, 8], [8, 16], ngroups=2)
    assert got == [3314076223, 1712484799]
