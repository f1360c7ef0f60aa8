"""GPU parity of the flat-stream ragged kernels (crc32_flat_prep/_kernel/_finish_kernel,
DESIGN.md §4): every checksum bit-exact against the oracle restatement of src/crc32.rs.

Layouts cover what the flat path must get right (packets crossing region ends, several
packets in one 128-B step, empty packets, the first packet at a 128-B boundary, gaps,
unaligned bases) and what it must hand to the sorted path (packets out of address
order, overlapping packets, gaps above 4 KiB, a packet spanning too many regions).
ENET_CRC_RAGGED=flatonly runs the flat kernels alone, so a correct result there is the
flat path's own; =flat (flat kernels with the streaming fallback) and the default mode
must match the oracle on every layout.
"""
import numpy as np
import pytest

import _oracle
from _data import ENET_SEED, packed_offsets, ragged_lengths, splitmix64_bytes

torch = pytest.importorskip("torch")
import rusty_enet_amd as rea  # noqa: E402

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    assert torch.cuda.is_available(), "GPU tests need a HIP device"
    return torch.device("cuda:0")


def run(data, offsets, lengths, dev, base_shift=0):
    d = torch.from_numpy(np.ascontiguousarray(data)).to(dev)
    if base_shift:
        d = d[base_shift:]
        offsets = offsets - np.uint64(base_shift)
    off = torch.from_numpy(offsets.astype(np.int64)).to(dev)
    ln = torch.from_numpy(lengths.astype(np.int32)).to(dev)
    out = rea.crc32_batch(d, offsets=off, lengths=ln)
    torch.cuda.synchronize()
    return out.cpu().numpy().view(np.uint32)


def with_gaps(lengths, gaps, start=0):
    offs = np.zeros(len(lengths), dtype=np.uint64)
    pos = start
    for i, (n, g) in enumerate(zip(lengths, gaps)):
        pos += int(g)
        offs[i] = pos
        pos += int(n)
    return offs, pos


def layout(name):
    rng = np.random.default_rng(abs(hash(name)) % (1 << 32))
    if name == "packed_enet":
        lengths = ragged_lengths(ENET_SEED + 21, 200_000)
        offsets = packed_offsets(lengths)
    elif name == "tiny_and_empty":  # several packets per step, empty ones everywhere
        lengths = rng.integers(0, 40, 60_000).astype(np.uint32)
        lengths[rng.random(60_000) < 0.2] = 0
        offsets = packed_offsets(lengths)
    elif name == "many_tiny":  # ~18 packets per region: many window switches in every group at once
        lengths = rng.integers(0, 64, 600_000).astype(np.uint32)
        offsets = packed_offsets(lengths) + np.uint64(9)
    elif name == "empty_first_at_boundary":  # empty packets at lo (128-aligned) and at step ends
        lengths = rng.integers(0, 300, 20_000).astype(np.uint32)
        lengths[:5] = 0
        lengths[1000:1010] = 0
        offsets = packed_offsets(lengths)
    elif name == "gaps_upto_4k":
        lengths = rng.integers(1, 1500, 30_000).astype(np.uint32)
        gaps = rng.integers(0, 4097, 30_000)
        offsets, _ = with_gaps(lengths, gaps, start=5)
    elif name == "receive_slots":  # fixed 1500-B slots, ragged datagrams (recvmmsg layout)
        lengths = rng.integers(20, 1500, 50_000).astype(np.uint32)
        offsets = np.arange(50_000, dtype=np.uint64) * np.uint64(1500)
    elif name == "long_packets":  # packets crossing several region ends (tail pieces)
        lengths = rng.integers(30_000, 70_000, 6000).astype(np.uint32)
        offsets = packed_offsets(lengths) + np.uint64(3)
    elif name == "mixed_lengths":
        lengths = np.concatenate([rng.integers(0, 64, 20_000), rng.integers(1000, 20_000, 2000),
                                  rng.integers(64, 1392, 20_000)]).astype(np.uint32)
        rng.shuffle(lengths)
        offsets = packed_offsets(lengths) + np.uint64(7)
    # --- layouts the flat path must refuse (default mode: sorted path) ---
    elif name == "shuffled_order":
        lengths = ragged_lengths(ENET_SEED + 22, 50_000)
        offsets = packed_offsets(lengths)
        perm = rng.permutation(50_000)
        lengths, offsets = lengths[perm], offsets[perm]
    elif name == "overlapping":
        lengths = rng.integers(100, 1400, 40_000).astype(np.uint32)
        offsets = np.cumsum(rng.integers(0, 90, 40_000)).astype(np.uint64)
    elif name == "gap_above_4k":
        lengths = rng.integers(1, 1500, 30_000).astype(np.uint32)
        gaps = np.zeros(30_000, dtype=np.int64)
        gaps[15_000] = 5000
        offsets, _ = with_gaps(lengths, gaps)
    elif name == "one_huge_packet":
        lengths = rng.integers(64, 1392, 8000).astype(np.uint32)
        lengths[4000] = 40 << 20
        offsets = packed_offsets(lengths)
    else:
        raise KeyError(name)
    end = int((offsets.astype(np.int64) + lengths.astype(np.int64)).max())
    data = splitmix64_bytes(len(name) * 7919 + 1, end + 64)
    return data, offsets.astype(np.uint64), lengths.astype(np.uint32)


FLAT = ["packed_enet", "tiny_and_empty", "many_tiny", "empty_first_at_boundary", "gaps_upto_4k", "receive_slots",
        "long_packets", "mixed_lengths"]
REFUSED = ["shuffled_order", "overlapping", "gap_above_4k", "one_huge_packet"]


@pytest.mark.parametrize("name", FLAT)
def test_flat_kernels_alone(dev, name, monkeypatch):
    monkeypatch.setenv("ENET_CRC_RAGGED", "flatonly")
    data, offsets, lengths = layout(name)
    assert np.array_equal(run(data, offsets, lengths, dev), _oracle.crc32_ragged(data, offsets, lengths))


@pytest.mark.parametrize("mode", ["flat", "default"])
@pytest.mark.parametrize("name", FLAT + REFUSED)
def test_every_layout(dev, name, mode, monkeypatch):
    if mode != "default":
        monkeypatch.setenv("ENET_CRC_RAGGED", mode)
    data, offsets, lengths = layout(name)
    assert np.array_equal(run(data, offsets, lengths, dev), _oracle.crc32_ragged(data, offsets, lengths))


@pytest.mark.parametrize("shift", [1, 2, 3, 5, 13, 64, 127])
def test_flat_unaligned_bases(dev, shift, monkeypatch):
    monkeypatch.setenv("ENET_CRC_RAGGED", "flatonly")
    lengths = ragged_lengths(ENET_SEED + 23 + shift, 20_000, lo=0, hi=2000)
    offsets = packed_offsets(lengths) + np.uint64(shift + 128)
    data = splitmix64_bytes(shift, int(offsets[-1]) + int(lengths[-1]) + 64)
    assert np.array_equal(run(data, offsets, lengths, dev, base_shift=shift),
                          _oracle.crc32_ragged(data, offsets, lengths))


def test_flat_matches_sorted_path_full_size(dev, monkeypatch):
    """G2 (1M x U[64,1392] packed): the flat kernels and the sorted path agree bit for bit."""
    lengths = ragged_lengths(ENET_SEED, 1 << 20)
    offsets = packed_offsets(lengths)
    g = torch.Generator(device=dev)
    g.manual_seed(ENET_SEED + 9)
    d = torch.randint(0, 256, (int(lengths.sum()),), dtype=torch.uint8, device=dev, generator=g)
    off = torch.from_numpy(offsets.astype(np.int64)).to(dev)
    ln = torch.from_numpy(lengths.astype(np.int32)).to(dev)
    monkeypatch.setenv("ENET_CRC_RAGGED", "flatonly")
    flat = rea.crc32_batch(d, offsets=off, lengths=ln)
    monkeypatch.setenv("ENET_CRC_RAGGED", "sorted")
    srt = rea.crc32_batch(d, offsets=off, lengths=ln)
    torch.cuda.synchronize()
    assert torch.equal(flat, srt)
