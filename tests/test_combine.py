"""Merged digest of a sharded batch: ``enet_crc32_combine``, a host
function of the C ABI (no device work), must give crc32(&[a, b]) from crc32(&[a]),
crc32(&[b]) and len(b), in the reference's output convention (src/crc32.rs:46), exactly
as the oracle restatement of src/crc32.rs:39-47 computes it over the concatenation.
"""
import numpy as np
import pytest

import _oracle
from _data import splitmix64_bytes

import rusty_enet_amd as rea


@pytest.mark.parametrize("seed", range(4))
def test_combine_matches_concatenation(seed):
    rng = np.random.default_rng(seed)
    for _ in range(200):
        la, lb = (int(rng.choice([0, 1, 3, 4, 5, 64, 1200, 1392, int(rng.integers(0, 9000))])) for _ in range(2))
        buf = splitmix64_bytes(int(rng.integers(1 << 62)), la + lb)
        a, b = buf[:la], buf[la:]
        ca, cb = _oracle.crc32([a]), _oracle.crc32([b])
        assert rea.crc32_combine(ca, cb, lb) == _oracle.crc32([a, b]) == _oracle.crc32([buf]), (la, lb)


def test_combine_reference_kats():
    # src/crc32.rs:52-55: [1..8] -> 3314076223 and [[1..8], [8..1]] -> 1712484799.
    a = np.arange(1, 9, dtype=np.uint8)
    b = a[::-1].copy()
    ca, cb = _oracle.crc32([a]), _oracle.crc32([b])
    assert ca == 3314076223
    assert rea.crc32_combine(ca, cb, len(b)) == 1712484799


def test_combine_shards_and_long_lengths():
    # The per-packet checksums of a batch fold into the digest of the whole buffer; and
    # the operator powering stays consistent far past any buffer we can hold:
    # combine(combine(A, B, nB), C, nC) == combine(A, combine(B, C, nC), nB + nC)
    # for lengths up to 2^63 (checks M8^(n1 + n2) = M8^n1 M8^n2 on every level).
    rng = np.random.default_rng(7)
    lengths = rng.integers(0, 3000, 64)
    buf = splitmix64_bytes(99, int(lengths.sum()))
    digest, off = None, 0
    for n in lengths:
        c = _oracle.crc32([buf[off:off + n]])
        digest = c if digest is None else rea.crc32_combine(digest, c, int(n))
        off += n
    assert digest == _oracle.crc32([buf])
    for _ in range(200):
        A, B, C = (int(x) for x in rng.integers(0, 1 << 32, 3, dtype=np.uint64))
        nb, nc = (int(x) for x in rng.integers(0, 1 << 62, 2, dtype=np.uint64))
        left = rea.crc32_combine(rea.crc32_combine(A, B, nb), C, nc)
        right = rea.crc32_combine(A, rea.crc32_combine(B, C, nc), nb + nc)
        assert left == right
    assert rea.crc32_combine(0x12345678, 0, 0) == 0x12345678


def test_combine_ladder_and_matrix_paths_agree():
    # Lengths below 2^34 take the host ladder (M32^(2^k) tables), longer ones the GF(2)
    # matrix powering: f(x, n) = combine(x, 0, n) must compose across the switch-over.
    rng = np.random.default_rng(11)
    for _ in range(100):
        x = int(rng.integers(0, 1 << 32, dtype=np.uint64))
        n1 = (1 << 34) - int(rng.integers(1, 4096))
        n2 = int(rng.integers(1, 8192))
        lhs = rea.crc32_combine(rea.crc32_combine(x, 0, n1), 0, n2)
        assert lhs == rea.crc32_combine(x, 0, n1 + n2), (n1, n2)
        assert rea.crc32_combine(rea.crc32_combine(x, 0, n2), 0, n1) == lhs
