"""Host model of the ragged jobs kernel's in-wave counting sort (crc32_kernels.hip, job_build).

One wave sorts a job of up to 256 packets (4 per lane, packet 4 lane + i) by step class
(min(nsteps, 15); positions past the job's n packets are not counted and keep their own index).
Class counts live in 4 words of 8-bit fields (class c: word c >> 2, field c & 3); the kernel scans
them over the lanes with wrapping 32-bit adds, reads the totals at lane 63, and forms each class's
first position with two multiplies per word.  A field can reach 256 (all 256 packets in one
class), and a sum of fields can carry into the next field, but only when every packet lies in that
class or below, so the carry only lands in classes that hold no packet.  This restates the exact
word arithmetic and checks that every packet lands on the position a stable sort by class gives
it, for random jobs and for the corner cases (one class holding all 256, partial jobs, the top
class of a word full).
"""
import random

import pytest

M = 0xFFFFFFFF
CLASSES, WORDS = 16, 4


def kernel_positions(cls, n):
    """cls[lane][i] (0..15, or 16 for no packet) -> the kernel's position of every packet."""
    cnt = [[0] * WORDS for _ in range(64)]
    rank = [[0] * 4 for _ in range(64)]
    for L in range(64):
        for i in range(4):
            c = cls[L][i]
            rank[L][i] = sum(1 for j in range(i) if cls[L][j] == c)
            one = (1 << (8 * (c & 3))) if c < CLASSES else 0
            for w in range(WORDS):
                cnt[L][w] = (cnt[L][w] + (one if (c >> 2) == w else 0)) & M
    start = [[0] * WORDS for _ in range(64)]
    run = 0
    for w in range(WORDS):
        acc = 0
        incl = []
        for L in range(64):  # wave_inclusive_add, wrapping
            acc = (acc + cnt[L][w]) & M
            incl.append(acc)
        tot = incl[63]
        base = (tot * 0x01010100 + (run & 255) * 0x01010101) & M
        run = (run + (((tot * 0x01010101) & M) >> 24)) & M
        for L in range(64):
            start[L][w] = (incl[L] - cnt[L][w] + base) & M
    pos = {}
    for L in range(64):
        for i in range(4):
            c = cls[L][i]
            if c < CLASSES:
                sw = start[L][c >> 2]
                pos[4 * L + i] = ((sw >> (8 * (c & 3))) & 255) + rank[L][i]
            else:
                pos[4 * L + i] = 4 * L + i
    return pos


def want_positions(cls, n):
    flat = [(cls[L][i], 4 * L + i) for L in range(64) for i in range(4)]
    valid = sorted((c, p) for c, p in flat if c < CLASSES)  # stable: by class, then packet index
    pos = {p: q for q, (_, p) in enumerate(valid)}
    for c, p in flat:
        if c >= CLASSES:
            pos[p] = p
    return pos


def job(classes_of_packets):
    n = len(classes_of_packets)
    full = list(classes_of_packets) + [CLASSES] * (256 - n)
    return [full[4 * L:4 * L + 4] for L in range(64)], n


def check(classes_of_packets):
    cls, n = job(classes_of_packets)
    got, want = kernel_positions(cls, n), want_positions(cls, n)
    assert got == want
    assert sorted(got.values()) == list(range(256))


@pytest.mark.parametrize("c", range(CLASSES))
def test_one_class_holds_the_whole_job(c):
    check([c] * 256)


@pytest.mark.parametrize("n", [0, 1, 7, 8, 127, 128, 200, 255, 256])
def test_partial_jobs(n):
    rng = random.Random(n)
    check([rng.randrange(CLASSES) for _ in range(n)])
    check([15] * n)
    check([3] * n)


def test_full_fields_next_to_packets():
    # a word's top class full up to the job's end, classes above it empty
    for c in (3, 7, 11):
        check([c - 1] * 6 + [c] * 250)
        check([0] * 1 + [c] * 255)
    # every class of one word, then nothing
    check(sorted([random.Random(5).randrange(4) for _ in range(256)]))
    # two classes of 128
    check([2] * 128 + [9] * 128)
    check([15] * 128 + [0] * 128)


def test_random_jobs():
    rng = random.Random(2026)
    for t in range(300):
        n = rng.choice([256, 256, 256, rng.randrange(257)])
        k = rng.choice([1, 2, 3, 16])
        pool = rng.sample(range(CLASSES), k)
        check([rng.choice(pool) for _ in range(n)])


def test_g2_like_jobs():
    # G2: lengths U[64, 1392] -> step classes 1..11
    rng = random.Random(7)
    for _ in range(50):
        check([min(15, ((rng.randint(64, 1392) + 3) // 4 + 3) // 4 // 8 + 1) for _ in range(256)])


def test_record_geometry_in_32_bit_words():
    """ragged_record's 32-bit nwords / nsteps / a1 equal make_geo's 64-bit ones (crc32_geometry.hpp)
    for every start phase and lengths up to 2^32 - 1."""
    rng = random.Random(11)
    lens = [0, 1, 2, 3, 4, 5, 127, 128, 129, 1392, 65536, (1 << 32) - 1, (1 << 32) - 2, (1 << 32) - 5, (1 << 32) - 6]
    lens += [rng.randrange(1 << 32) for _ in range(2000)]
    for ln in lens:
        for sa in (0x7F0000000000 + p for p in range(4)):
            z = (4 - (sa + ln) % 4) % 4 if ln else 0
            ea = sa + ln + z
            top, a1 = sa & ~3, ea & ~3
            nwords = (a1 - top) >> 2
            nsteps = ((nwords + 3) // 4 + 7) // 8
            v = sa & 3
            nw32 = ((ln >> 2) + (((ln & 3) + v + z) >> 2)) & M
            ns32 = ((((nw32 + 3) & M) >> 2) + 7) >> 3
            assert (nw32, ns32, top + 4 * nw32) == (nwords, nsteps, a1), (ln, sa)
            assert (128 * ns32 - 4 * nw32) & M == 128 * nsteps - 4 * nwords < 128
