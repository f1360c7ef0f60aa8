"""GPU parity of the pinned receive ring: datagrams written straight
into pinned slot memory, checksummed per slot with copies and kernels overlapped, bit-exact
against the oracle; slot reuse, in-flight protection and descriptor validation."""
import ctypes

import numpy as np
import pytest

import _oracle
from _data import packed_offsets, ragged_lengths, splitmix64_bytes

torch = pytest.importorskip("torch")
from rusty_enet_amd import _native  # noqa: E402
from rusty_enet_amd.ring import ReceiveRing  # noqa: E402

pytestmark = pytest.mark.gpu


def fill(ring, i, seed, n, lo=0, hi=1400):
    data, off, ln, _ = ring.slot(i)
    lengths = ragged_lengths(seed, n, lo=lo, hi=hi)
    offsets = packed_offsets(lengths) + np.uint64(i % 3)  # unaligned starts too
    total = int(offsets[-1] + lengths[-1]) if n else 0
    data[:total] = splitmix64_bytes(seed + 1, total)
    off[:n] = offsets
    ln[:n] = lengths
    return _oracle.crc32_ragged(data[:max(total, 1)].copy(), offsets, lengths)


def test_ring_slots_bit_exact_and_reusable():
    assert torch.cuda.is_available()
    with ReceiveRing(0, nslots=3, slot_bytes=8 << 20, slot_packets=8192) as ring:
        want = {}
        for rnd in range(3):  # every slot is reused: no stale results
            counts = [8192, 300 + rnd, 5000]
            for i, n in enumerate(counts):
                want[i] = fill(ring, i, 1000 * rnd + i, n)
                ring.submit(i, n)
            for i, n in enumerate(counts):
                ring.wait(i)
                assert np.array_equal(ring.slot(i)[3][:n], want[i]), (rnd, i)


def test_ring_validation_and_in_flight():
    with ReceiveRing(0, nslots=2, slot_bytes=1 << 20, slot_packets=4096) as ring:
        fill(ring, 0, 7, 4096, hi=200)
        ring.submit(0, 4096)
        with pytest.raises(_native.CrcError):
            ring.submit(0, 1)  # in flight
        ring.wait(0)
        ring.wait(0)  # idempotent
        with pytest.raises(_native.CrcError):
            ring.submit(0, 4097)  # more packets than the slot holds
        _, off, ln, _ = ring.slot(1)
        off[0], ln[0] = (1 << 20) - 10, 11  # one byte past the slot
        with pytest.raises(_native.CrcError):
            ring.submit(1, 1)
        ring.submit(1, 0)  # empty submit is fine
        ring.wait(1)
