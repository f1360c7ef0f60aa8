"""GPU parity: every checksum from the gfx950 kernels (through the C ABI) is
bit-exact against the oracle restatement of src/crc32.rs and the zlib golden
fixtures.  Run on an MI355X with  python -m pytest tests -m gpu.
"""
import zlib

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


def as_u32(t) -> np.ndarray:
    return t.cpu().numpy().view(np.uint32)


def to_dev(a: np.ndarray, dev):
    return torch.from_numpy(np.ascontiguousarray(a)).to(dev)


def ragged_on_device(data, offsets, lengths, dev):
    d = to_dev(data, dev)
    off = to_dev(offsets.astype(np.int64), dev)
    ln = to_dev(lengths.astype(np.int32), dev)
    out = rea.crc32_batch(d, offsets=off, lengths=ln)
    torch.cuda.synchronize()
    return as_u32(out)


# --- the reference's own tests, through the per-call drop-in (enet_crc32_iov) ----

def test_reference_kats_per_call(dev):
    assert rea.crc32([bytes([1, 2, 3, 4, 5, 6, 7, 8])]) == 3314076223          # src/crc32.rs:52
    assert rea.crc32([bytes([1, 2, 3, 4, 5, 6, 7, 8]),
                      bytes([8, 7, 6, 5, 4, 3, 2, 1])]) == 1712484799          # src/crc32.rs:54-55


def test_golden_kats_per_call(dev, golden):
    ctx = rea.default_context(0)
    for k in golden["kat"]:
        assert ctx([bytes(s) for s in k["slices_bytes"]]) == k["expected"], k["name"]


def test_golden_cases_per_call(dev, golden):
    ctx = rea.default_context(0)
    for case in golden["cases"]:
        slices = [splitmix64_bytes(s, n) for s, n in case["slices"]]
        assert ctx(slices) == case["expected"], case["name"]


def test_golden_cases_in_one_ragged_batch(dev, golden):
    # Every golden input concatenated, placed at deliberately misaligned offsets.
    blobs = [b"".join(bytes(splitmix64_bytes(s, n)) for s, n in c["slices"]) for c in golden["cases"]]
    offsets, pos, parts = [], 3, [b"\xAA" * 3]
    for i, b in enumerate(blobs):
        offsets.append(pos)
        parts.append(b)
        gap = i % 5
        parts.append(b"\x55" * gap)
        pos += len(b) + gap
    data = np.frombuffer(b"".join(parts) + b"\x00" * 16, dtype=np.uint8)
    got = ragged_on_device(data, np.array(offsets, dtype=np.uint64),
                           np.array([len(b) for b in blobs], dtype=np.uint32), dev)
    want = np.array([c["expected"] for c in golden["cases"]], dtype=np.uint32)
    assert np.array_equal(got, want)


# --- exhaustive small shapes ------------------------------------------------------

def test_every_length_every_alignment(dev):
    # lengths 0..700 at start offsets 0..15 (both the 4-byte grid and the 16-byte
    # chunking see every phase), packed back to back.
    lens, offs, pos = [], [], 0
    for n in range(0, 701):
        for a in range(16):
            pos += a  # gap -> start phase varies
            offs.append(pos)
            lens.append(n)
            pos += n
    data = splitmix64_bytes(11, pos + 64)
    offsets = np.array(offs, dtype=np.uint64)
    lengths = np.array(lens, dtype=np.uint32)
    got = ragged_on_device(data, offsets, lengths, dev)
    assert np.array_equal(got, _oracle.crc32_ragged(data, offsets, lengths))


def test_uniform_batch_1200(dev):
    n, L = 65536, 1200
    data = splitmix64_bytes(ENET_SEED, n * L)
    d = to_dev(data, dev)
    got = as_u32(rea.crc32_batch(d, stride=L, length=L, count=n))
    assert np.array_equal(got, _oracle.crc32_uniform(data, L, L, n, threads=8))


@pytest.mark.parametrize("stride,length", [(1201, 1200), (1392, 1392), (1396, 1393), (64, 64), (7, 5), (4096, 4096)])
def test_uniform_batch_shapes(dev, stride, length):
    n = 20000
    data = splitmix64_bytes(stride * 31 + length, (n - 1) * stride + length)
    d = to_dev(data, dev)
    got = as_u32(rea.crc32_batch(d, stride=stride, length=length, count=n))
    assert np.array_equal(got, _oracle.crc32_uniform(data, stride, length, n, threads=8))


def test_large_buffers_64k(dev):
    n, L = 256, 65536
    data = splitmix64_bytes(77, n * L)
    d = to_dev(data, dev)
    got = as_u32(rea.crc32_batch(d, stride=L, length=L, count=n))
    assert np.array_equal(got, _oracle.crc32_uniform(data, L, L, n, threads=8))


def test_large_unaligned_odd_lengths(dev):
    lengths = np.array([65536 + 3, 100000, 1, 0, 262147, 4095, 70001], dtype=np.uint32)
    offsets = packed_offsets(lengths) + np.uint64(1)
    data = splitmix64_bytes(78, int(lengths.sum()) + 8)
    got = ragged_on_device(data, offsets, lengths, dev)
    assert np.array_equal(got, _oracle.crc32_ragged(data, offsets, lengths))


# --- BASELINE.json full-size configs ------------------------------------------------

def test_full_size_uniform_1m_x_1200(dev):
    n, L = 1 << 20, 1200
    g = torch.Generator(device=dev)
    g.manual_seed(ENET_SEED)
    d = torch.randint(0, 256, (n * L,), dtype=torch.uint8, device=dev, generator=g)
    got = as_u32(rea.crc32_batch(d, stride=L, length=L, count=n))
    want = _oracle.crc32_uniform(d.cpu().numpy(), L, L, n, threads=16)
    assert np.array_equal(got, want)


def test_full_size_ragged_1m(dev):
    lengths = ragged_lengths(ENET_SEED, 1 << 20)
    offsets = packed_offsets(lengths)
    total = int(lengths.sum())
    g = torch.Generator(device=dev)
    g.manual_seed(ENET_SEED + 1)
    d = torch.randint(0, 256, (total,), dtype=torch.uint8, device=dev, generator=g)
    out = rea.crc32_batch(d, offsets=to_dev(offsets.astype(np.int64), dev),
                          lengths=to_dev(lengths.astype(np.int32), dev))
    got = as_u32(out)
    assert np.array_equal(got, _oracle.crc32_ragged(d.cpu().numpy(), offsets, lengths))


@pytest.mark.parametrize("layout", ["line_aligned", "packed_base_3"])
def test_full_size_ragged_layouts(dev, layout):
    """G2's 1M datagrams in the two other layouts round 5 measured: every datagram starting
    on a 128-B line (scripts/exp_layout.py, the over-fetch A/B) and packed from
    a buffer base 3 bytes past a line (every top chunk unaligned, the batch's first round near
    the base); all checksums against the oracle (16 threads)."""
    lengths = ragged_lengths(ENET_SEED, 1 << 20)
    if layout == "line_aligned":
        stride = (lengths.astype(np.uint64) + 127) // 128 * 128
        offsets = np.concatenate([[0], np.cumsum(stride)[:-1]]).astype(np.uint64)
    else:
        offsets = packed_offsets(lengths) + np.uint64(3)
    total = int(offsets[-1]) + int(lengths[-1])
    g = torch.Generator(device=dev)
    g.manual_seed(ENET_SEED + 21)
    d = torch.randint(0, 256, (total,), dtype=torch.uint8, device=dev, generator=g)
    got = as_u32(rea.crc32_batch(d, offsets=to_dev(offsets.astype(np.int64), dev),
                                 lengths=to_dev(lengths.astype(np.int32), dev)))
    want = _oracle.crc32_ragged(d.cpu().numpy(), offsets, lengths, threads=16)
    del d
    assert np.array_equal(got, want), int(np.count_nonzero(got != want))


def test_kernels_agree_on_the_same_bytes(dev):
    """HIP against HIP: the same packets through the uniform kernels (stride form) and the
    ragged jobs kernel (offsets / lengths form) give the same checksums, for G1's 1200-B
    packets (whole-line kernel), 1393-B packets at an odd stride (register ring) and 64-KiB
    buffers (wave-per-packet kernel); both are also checked in full against the oracle, so the
    agreement is never the only evidence."""
    for n, stride, L, seed in ((1 << 18, 1200, 1200, 91), (1 << 16, 1396, 1393, 92), (512, 65536, 65536, 93)):
        g = torch.Generator(device=dev)
        g.manual_seed(seed)
        d = torch.randint(0, 256, ((n - 1) * stride + L,), dtype=torch.uint8, device=dev, generator=g)
        uni = as_u32(rea.crc32_batch(d, stride=stride, length=L, count=n))
        offsets = np.arange(n, dtype=np.int64) * stride
        rag = as_u32(rea.crc32_batch(d, offsets=to_dev(offsets, dev),
                                     lengths=to_dev(np.full(n, L, dtype=np.int32), dev)))
        assert np.array_equal(uni, rag), (stride, L)
        want = _oracle.crc32_uniform(d.cpu().numpy(), stride, L, n, threads=16)
        assert np.array_equal(uni, want), (stride, L)


def test_full_shard_uniform_2m_x_1200(dev):
    """The per-GPU shard of configs[3] (16M x 1200 B over 8 GPUs): 2M x 1200 B = 2.4 GB."""
    n, L = 2 << 20, 1200
    g = torch.Generator(device=dev)
    g.manual_seed(ENET_SEED + 3)
    d = torch.randint(0, 256, (n * L,), dtype=torch.uint8, device=dev, generator=g)
    got = as_u32(rea.crc32_batch(d, stride=L, length=L, count=n))
    want = _oracle.crc32_uniform(d.cpu().numpy(), L, L, n, threads=16)
    del d
    assert np.array_equal(got, want)


def test_full_shard_large_32768_x_64k(dev):
    """The per-GPU shard of configs[4] (256K x 64 KiB over 8 GPUs): 32768 x 64 KiB = 2 GiB."""
    n, L = 32768, 65536
    g = torch.Generator(device=dev)
    g.manual_seed(ENET_SEED + 4)
    d = torch.randint(0, 256, (n * L,), dtype=torch.uint8, device=dev, generator=g)
    got = as_u32(rea.crc32_batch(d, stride=L, length=L, count=n))
    want = _oracle.crc32_uniform(d.cpu().numpy(), L, L, n, threads=16)
    del d
    assert np.array_equal(got, want)


@pytest.mark.parametrize("base", [0, 1, 3, 100])
def test_full_size_frag_64k_datagrams(dev, base):
    """the configs[4] bytes as the reference checksums them (bench.py's
    `frag_64k`): 32,768 payloads of 64 KiB, each fragmented at the default MTU into 48
    datagrams of 1392 B and one of 288 B (src/c/peer.rs:181-192), packed back to back from
    `base`: all 1,605,632 datagrams against the oracle (16 threads).  Since round 6 their
    1392-B rounds are line rounds (bases 0, +1, +3)."""
    n = 32768
    lengths = np.tile(np.array([1392] * 48 + [288], dtype=np.uint32), n)
    offsets = packed_offsets(lengths) + np.uint64(base)
    total = int(lengths.sum()) + base
    g = torch.Generator(device=dev)
    g.manual_seed(ENET_SEED + 5 + base)
    d = torch.randint(0, 256, (total,), dtype=torch.uint8, device=dev, generator=g)
    got = as_u32(rea.crc32_batch(d, offsets=to_dev(offsets.astype(np.int64), dev),
                                 lengths=to_dev(lengths.astype(np.int32), dev)))
    want = _oracle.crc32_ragged(d.cpu().numpy(), offsets, lengths, threads=16)
    del d
    assert got.size == lengths.size == 1_605_632
    assert np.array_equal(got, want), int(np.count_nonzero(got != want))


# --- properties --------------------------------------------------------------------

def test_single_bit_flips_are_detected(dev):
    # The CRC is the corruption detector of src/c/protocol.rs:1499-1501: every
    # single-bit error in a datagram must change its checksum.
    n, L = 4096, 1200
    data = splitmix64_bytes(5, n * L)
    d = to_dev(data, dev)
    base = as_u32(rea.crc32_batch(d, stride=L, length=L, count=n))
    rng = np.random.default_rng(0)
    pos = np.arange(n) * L + rng.integers(0, L, n)
    bits = rng.integers(0, 8, n)
    flipped = data.copy()
    flipped[pos] ^= (1 << bits).astype(np.uint8)
    got = as_u32(rea.crc32_batch(to_dev(flipped, dev), stride=L, length=L, count=n))
    assert np.all(got != base)
    assert np.array_equal(got, _oracle.crc32_uniform(flipped, L, L, n, threads=8))


def test_repeatable_and_stream_ordered(dev):
    n, L = 50000, 1200
    data = to_dev(splitmix64_bytes(6, n * L), dev)
    s = torch.cuda.Stream(device=dev)
    with torch.cuda.stream(s):
        a = rea.crc32_batch(data, stride=L, length=L, count=n, stream=s)
        b = rea.crc32_batch(data, stride=L, length=L, count=n, stream=s)
    s.synchronize()
    assert torch.equal(a, b)
    # and both equal the oracle (a repeat of a wrong answer would pass the comparison above)
    want = _oracle.crc32_uniform(data.cpu().numpy(), L, L, n, threads=16)
    assert np.array_equal(as_u32(a), want)


def test_empty_batch_and_zero_length(dev):
    d = torch.zeros(16, dtype=torch.uint8, device=dev)
    out = rea.crc32_batch(d, stride=0, length=0, count=5)
    assert np.array_equal(as_u32(out), np.zeros(5, dtype=np.uint32))  # crc32(&[]) == 0
    out = rea.crc32_batch(d, stride=16, length=16, count=0)
    assert out.numel() == 0


def test_host_batch_end_to_end(dev):
    lengths = ragged_lengths(9, 300000)
    offsets = packed_offsets(lengths) + np.uint64(2)
    data = splitmix64_bytes(10, int(lengths.sum()) + 8)
    ctx = rea.Context(0)
    got = ctx.crc32_ragged_host(data, offsets, lengths)
    ctx.close()
    assert np.array_equal(got, _oracle.crc32_ragged(data, offsets, lengths))


def test_per_call_65_slices(dev):
    # The send path passes a 65-slice array (BUFFER_MAXIMUM), most of them empty.
    rng = np.random.default_rng(3)
    for trial in range(20):
        slices = [splitmix64_bytes(100 * trial + j, int(rng.integers(0, 40)) if j < 9 else 0) for j in range(65)]
        assert rea.crc32(slices) == _oracle.crc32(slices)


# --- region sort (default ragged pre-pass): region sizes and grids around its edges ----------

@pytest.mark.parametrize("count", [4096, 4100, 5000, 8 * 4096 + 3, 70_001])
def test_ragged_region_sort_edges(dev, count):
    # 4096: the smallest sorted batch; 4100: a grid of 33 workgroups (not a multiple of 8,
    # so 4096-packet regions and the plain round order); 5000: 40 workgroups (XCD-aligned
    # regions of 640); the others end in a partial region and a partial round.  Lengths
    # 0..3000 so every region mixes step classes (empty packets included), unaligned starts.
    rng = np.random.default_rng(count)
    lengths = rng.integers(0, 3001, size=count).astype(np.uint32)
    lengths[rng.integers(0, count, size=count // 50)] = 0
    gaps = rng.integers(0, 4, size=count).astype(np.uint64)
    offsets = (packed_offsets(lengths) + np.cumsum(gaps)).astype(np.uint64) + np.uint64(3)
    data = splitmix64_bytes(count + 1, int(offsets[-1] + lengths[-1]) + 8)
    assert np.array_equal(ragged_on_device(data, offsets, lengths, dev), _oracle.crc32_ragged(data, offsets, lengths))


@pytest.mark.parametrize("zero_frac", [0.08, 0.3])
def test_ragged_empty_rounds(dev, zero_frac):
    # Jobs whose first rounds hold only empty packets (no fast body: the generic loop), next to
    # fast, line and generic rounds (packed and raw records); 64 of them in one batch.
    count = 64 * 136 + 5
    rng = np.random.default_rng(int(zero_frac * 100))
    lengths = rng.choice(np.array([0, 1, 100, 700, 1100, 1392, 1800, 2500, 3000], dtype=np.uint32), size=count)
    lengths[rng.random(count) < zero_frac] = 0
    lengths[:40] = 0
    offsets = (packed_offsets(lengths) + np.cumsum(rng.integers(0, 3, size=count))).astype(np.uint64)
    data = splitmix64_bytes(count + 7, int(offsets[-1] + lengths[-1]) + 8)
    assert np.array_equal(ragged_on_device(data, offsets, lengths, dev), _oracle.crc32_ragged(data, offsets, lengths))


@pytest.mark.parametrize("shape", ["near_base", "wide_spread", "tiny", "long_mix", "mtu_unaligned", "one_job"])
def test_ragged_round_paths(dev, shape):
    """The round bodies of crc32_ragged_jobs_kernel (8 packets per round, 128-B steps; first
    written for the parked 16-packet kernel): near_base: overlapping packets starting in the
    first 16 bytes of the buffer (top chunks that would reach below it: the generic body's
    fallback loads); wide_spread: six step classes far apart, so the rounds where classes
    meet differ by > 1 step (generic body); tiny: packets of <= 3 steps at every alignment
    (ring-length rounds, top slots 0, 1 and 2 mixed in one unrolled body); long_mix: packets
    of 15+ steps (the longer class, generic) next to short ones; mtu_unaligned: 1392-B
    datagrams from base + 1 (the frag_64k shape); one_job: a batch of one partial job per
    workgroup."""
    rng = np.random.default_rng(zlib.crc32(shape.encode()))
    n = 9000
    if shape == "near_base":
        lengths = rng.integers(0, 1500, size=n).astype(np.uint32)
        offsets = rng.integers(0, 16, size=n).astype(np.uint64)
        data = splitmix64_bytes(61, 16 + 1500 + 8)
    else:
        if shape == "wide_spread":
            lengths = rng.choice(np.array([40, 300, 560, 820, 1080, 1340], dtype=np.uint32), size=n)
        elif shape == "tiny":
            lengths = rng.integers(0, 193, size=n).astype(np.uint32)
        elif shape == "long_mix":
            lengths = np.where(rng.random(n) < 0.5, rng.integers(1400, 4097, size=n),
                               rng.integers(0, 200, size=n)).astype(np.uint32)
        elif shape == "mtu_unaligned":
            lengths = np.full(n, 1392, dtype=np.uint32)
        else:
            n = 4096 + 17
            lengths = rng.integers(0, 1500, size=n).astype(np.uint32)
        gaps = rng.integers(0, 5, size=n).astype(np.uint64) if shape in ("tiny", "long_mix") else np.zeros(n, np.uint64)
        offsets = (packed_offsets(lengths) + np.cumsum(gaps)).astype(np.uint64) + np.uint64(1)
        data = splitmix64_bytes(62, int(offsets[-1] + lengths[-1]) + 8)
    got = ragged_on_device(data, offsets, lengths, dev)
    want = _oracle.crc32_ragged(data, offsets, lengths)
    assert np.array_equal(got, want), int(np.count_nonzero(got != want))


@pytest.mark.parametrize("mix", ["adjacent_classes", "empties_in_short_rounds", "class_pairs_every_round"])
def test_ragged_mixed_class_rounds(dev, mix):
    """Rounds whose packets' top slots differ, all in the unrolled bodies since round 4
    (round_from_record: top slots in B .. B + 1, any in ring-length rounds):
    adjacent_classes: lengths at both sides of 128-B step boundaries, so sorted rounds straddle
    two classes (top slots 0 and 1) at every alignment; empties_in_short_rounds: zero-length
    packets among 1-3-step ones (ring-length rounds whose empty groups never read);
    class_pairs_every_round: 4 packets of each of two adjacent classes per 8, so nearly every
    round mixes (plus a few 3-class rounds, the generic body)."""
    rng = np.random.default_rng(zlib.crc32(mix.encode()))
    n = 12000
    if mix == "adjacent_classes":
        edge = rng.integers(2, 11, size=n) * 128
        lengths = (edge + rng.integers(-20, 21, size=n)).astype(np.uint32)
    elif mix == "empties_in_short_rounds":
        lengths = np.where(rng.random(n) < 0.3, 0, rng.integers(1, 384, size=n)).astype(np.uint32)
    else:
        pair = rng.integers(1, 10, size=n // 8)
        lengths = np.concatenate([np.concatenate([rng.integers(128 * p - 100, 128 * p + 1, size=4),
                                                  rng.integers(128 * p + 1, 128 * p + 100, size=4)])
                                  for p in pair]).astype(np.uint32)
    offsets = (packed_offsets(lengths) + np.cumsum(rng.integers(0, 4, size=lengths.size))).astype(np.uint64)
    offsets += np.uint64(2)
    data = splitmix64_bytes(63 + len(mix), int(offsets[-1] + lengths[-1]) + 8)
    got = ragged_on_device(data, offsets, lengths, dev)
    want = _oracle.crc32_ragged(data, offsets, lengths)
    assert np.array_equal(got, want), int(np.count_nonzero(got != want))


@pytest.mark.parametrize("shape", ["every_step_count", "every_phase_and_gap", "lines_and_ends_mixed",
                                   "job_boundaries", "overlapping"])
def test_ragged_line_rounds(dev, shape):
    """Line rounds (round 6, line_round_from_record; host model tests/test_line_rounds_model.py):
    rounds of 8 packets of one step count 8..13 run on whole 128-B lines.  every_step_count:
    each count 8..13 with every start phase 0..127 (so every 16-B end chunk j_last, every
    grid offset r and every first-word phase); every_phase_and_gap: one length per run of 8,
    random gaps (packets not back to back); lines_and_ends_mixed: line-eligible runs next to
    mixed-class and short rounds in the same jobs; job_boundaries: runs of 8 equal step
    counts that straddle 256-packet jobs, batch ends inside a run (a partial last round is
    never a line round); overlapping: the same bytes checksummed twice by packets of
    different rounds."""
    rng = np.random.default_rng(zlib.crc32(shape.encode()) + 6)
    if shape == "every_step_count":
        lengths, gaps = [], []
        for n in range(8, 14):
            for ph in range(128):
                ln = int(rng.integers(128 * (n - 1) + 5, 128 * n - 8))
                lengths += [ln] * 8
                gaps += [ph % 7] * 8
        lengths, gaps = np.array(lengths, dtype=np.uint32), np.array(gaps, dtype=np.uint64)
    elif shape == "every_phase_and_gap":
        runs = rng.integers(950, 1700, size=1024)
        lengths = np.repeat(runs, 8).astype(np.uint32)
        gaps = rng.integers(0, 64, size=lengths.size).astype(np.uint64)
    elif shape == "lines_and_ends_mixed":
        lengths = np.where(rng.random(16384) < 0.6, 1392, rng.integers(0, 1600, size=16384)).astype(np.uint32)
        gaps = rng.integers(0, 3, size=lengths.size).astype(np.uint64)
    elif shape == "job_boundaries":
        lengths = np.repeat(rng.integers(1000, 1700, size=1500), 8)[:4096 * 3 + 5].astype(np.uint32)
        gaps = np.zeros(lengths.size, dtype=np.uint64)
    else:
        lengths = np.full(8192, 1300, dtype=np.uint32)
        gaps = np.zeros(lengths.size, dtype=np.uint64)
    offsets = (packed_offsets(lengths) + np.cumsum(gaps)).astype(np.uint64) + np.uint64(int(rng.integers(0, 128)))
    if shape == "overlapping":
        offsets = (offsets // np.uint64(2)).astype(np.uint64)  # every byte read by two packets
    data = splitmix64_bytes(64 + len(shape), int(offsets.max() + lengths.max()) + 8)
    got = ragged_on_device(data, offsets, lengths, dev)
    want = _oracle.crc32_ragged(data, offsets, lengths)
    assert np.array_equal(got, want), int(np.count_nonzero(got != want))


# seeds chosen so that every draw kind (0-5) runs with and without overlapping packets
@pytest.mark.parametrize("seed", [102, 136, 103, 172, 130, 129, 105, 107, 114, 115, 100, 101])
def test_ragged_random_sweep(dev, seed):
    """The randomized ragged sweep (scripts/fuzz_ragged.py: 120 batches / 18.0 M datagrams
    bit-exact in round 5) as a regression guard: twelve seeded batches, each drawing a count,
    a length distribution (uniform ranges, MTU fragments with short tails, tiny, bimodal,
    128-B step edges, a long tail to 8 KiB; 2 % zero-length), gaps, overlapping re-reads and
    a base offset 0-15, checked in full against the oracle."""
    import importlib.util
    import os

    spec = importlib.util.spec_from_file_location(
        "fuzz_ragged", os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "scripts",
                                    "fuzz_ragged.py"))
    fz = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(fz)
    rng = np.random.default_rng(seed)
    kind, base, starts, lengths = fz.draw(rng)
    if lengths.size > 120_000:  # keep the suite fast: the draw's own distribution, fewer packets
        starts, lengths = starts[:120_000], lengths[:120_000]
    total = int((starts + lengths.astype(np.uint64)).max()) + base + 8
    data = rng.integers(0, 256, size=total, dtype=np.uint8)
    got = ragged_on_device(data[base:], starts, lengths, dev)
    want = _oracle.crc32_ragged(data[base:], starts, lengths, threads=8)
    assert np.array_equal(got, want), (kind, base, int(np.count_nonzero(got != want)))


# --- round-record scratch cached per stream (launch_ragged) ----------------------------------

def test_ragged_scratch_per_stream(dev):
    # Two streams, each launching sorted ragged batches that grow (the cached buffer is
    # regrown stream-ordered) and shrink (reused), interleaved without synchronising in
    # between; every result is kept and checked afterwards.
    streams = [torch.cuda.Stream(dev), torch.cuda.Stream(dev)]
    jobs = []
    for i, count in enumerate([5000, 40_000, 9000, 120_000, 4096, 70_000]):
        lengths = ragged_lengths(ENET_SEED + 40 + i, count, lo=0, hi=1500)
        offsets = packed_offsets(lengths) + np.uint64(i)
        data = splitmix64_bytes(40 + i, int(lengths.sum()) + 16)
        s = streams[i % 2]
        with torch.cuda.stream(s):
            d = to_dev(data, dev)
            off = to_dev(offsets.astype(np.int64), dev)
            ln = to_dev(lengths.astype(np.int32), dev)
            out = rea.crc32_batch(d, offsets=off, lengths=ln, stream=s)
        jobs.append((out, data, offsets, lengths, d, off, ln))
    torch.cuda.synchronize()
    for out, data, offsets, lengths, *_ in jobs:
        assert np.array_equal(as_u32(out), _oracle.crc32_ragged(data, offsets, lengths))


# --- whole-line loads: line-split register ring, non-temporal long packets -----------------

@pytest.mark.parametrize("base_off", [0, 4, 12, 16, 48, 100, 124])
def test_uniform_line_split_bases(dev, base_off):
    # Packet ends at every 16-B residue mod 128 (lo = 0..7 lanes taking entry s + 1),
    # lengths that are and are not multiples of 16, the first packets within a chunk of
    # the base (fallback loads), and a batch that ends exactly at the buffer's end.
    for stride, length, n in [(1200, 1200, 3001), (1392, 1392, 2999), (1204, 1200, 2048), (16, 16, 5000),
                              (132, 128, 4000), (1796, 1792, 1500), (400, 396, 3333)]:
        data = splitmix64_bytes(base_off * 7 + stride + length, base_off + (n - 1) * stride + length)
        d = to_dev(data, dev)[base_off:]
        got = as_u32(rea.crc32_batch(d, stride=stride, length=length, count=n))
        want = _oracle.crc32_uniform(data[base_off:], stride, length, n, threads=8)
        assert np.array_equal(got, want), (stride, length, base_off)


@pytest.mark.parametrize("base_off", [0, 128, 384, 4096])
def test_uniform_whole_lines_kernel(dev, base_off):
    # Back-to-back packets of 16-B multiple lengths from a line-aligned base: the whole-line
    # kernel (every line read once; group g's lines [g L / 128, (g+1) L / 128)) for every
    # whole round, the register ring for the < 8 packets left.  Lengths 528..1792 (5..14
    # lines per group slot), every j residue pattern, counts with and without a tail.
    for length, n in [(528, 8), (528, 4099), (640, 3000), (1040, 1001), (1200, 8), (1200, 9), (1200, 4007),
                      (1216, 777), (1280, 2048), (1392, 3007), (1504, 1600), (1776, 777), (1792, 1499)]:
        data = splitmix64_bytes(base_off * 5 + length + n, base_off + n * length)
        d = to_dev(data, dev)[base_off:]
        assert d.data_ptr() % 128 == 0
        got = as_u32(rea.crc32_batch(d, stride=length, length=length, count=n))
        want = _oracle.crc32_uniform(data[base_off:], length, length, n, threads=8)
        assert np.array_equal(got, want), (length, n, base_off, int(np.count_nonzero(got != want)))


@pytest.mark.parametrize("base_off", [16, 48, 80, 112, 8, 1040])
def test_uniform_whole_lines_head_peeled(dev, base_off):
    # Back-to-back 16-B-multiple packets from a 16-B aligned base that is not line-aligned:
    # the packets before the first one that starts on a line go through the register ring,
    # the whole-line kernel takes the whole rounds from there (launch_uniform, lines_shape).
    # Counts below, at and past the head, with and without a tail; 1280-B packets never
    # start on a line from these bases, and base + 8 is not 16-B aligned (register ring).
    for length, n in [(1200, 3), (1200, 9), (1200, 15), (1200, 4011), (1392, 2999), (528, 4100), (1040, 1111),
                      (1280, 1000), (1792, 1501)]:
        data = splitmix64_bytes(base_off * 3 + length + n, base_off + n * length)
        d = to_dev(data, dev)[base_off:]
        got = as_u32(rea.crc32_batch(d, stride=length, length=length, count=n))
        want = _oracle.crc32_uniform(data[base_off:], length, length, n, threads=8)
        assert np.array_equal(got, want), (length, n, base_off, int(np.count_nonzero(got != want)))


def test_long_packets_line_ends(dev):
    # Non-temporal DMAs need every packet to end on a 128-B line: ends aligned with the
    # starts aligned (64 KiB from an aligned base) or not (65536 - 128 from base + 128),
    # and a base that breaks the line ends (the plain path).
    # 1920 and 3968 B (15 and 31 steps): the 8-packets-per-wave DMA kernel, with and
    # without the hint; 2000 B from base + 4: that kernel without it.
    for base_off, stride, length, n in [(0, 65536, 65536, 64), (128, 65536, 65408, 64), (4, 65536, 65536, 48),
                                        (256, 8192, 4096, 300), (0, 1920, 1920, 5000), (0, 3968, 3968, 1000),
                                        (4, 1920, 1920, 4000), (4, 2000, 2000, 3000), (0, 4092, 4090, 999)]:
        data = splitmix64_bytes(base_off + length, base_off + (n - 1) * stride + length)
        d = to_dev(data, dev)[base_off:]
        got = as_u32(rea.crc32_batch(d, stride=stride, length=length, count=n))
        want = _oracle.crc32_uniform(data[base_off:], stride, length, n, threads=8)
        assert np.array_equal(got, want), (base_off, stride, length)


@pytest.mark.parametrize("base_off", [0, 4, 12, 128, 1000])
def test_long_packets_wave_kernel(dev, base_off):
    # One wave per packet, 1-KiB steps (crc32_wave_dma_kernel).
    # Lengths from the 4-KiB minimum up, multiples of 1 KiB and 128 B or not, odd lengths
    # (bytes past the end masked), gaps between packets, packets within a chunk of the
    # base (fallback loads), counts that are not multiples of the wave count.
    # Packets of a multiple of 8 KiB steps take the register-ring form (crc32_wave_regs_kernel),
    # the others the LDS-DMA ring.
    for stride, length, n in [(65536, 65536, 200), (4096, 4096, 3001), (4100, 4097, 999), (5000, 4999, 777),
                              (12288, 10001, 300), (65540, 65537, 33), (70000, 65536, 17), (8192, 8191, 1),
                              (4096, 4096, 4097), (32768, 32768, 501), (24580, 24573, 333), (16384, 16381, 1025)]:
        data = splitmix64_bytes(base_off * 3 + stride + length, base_off + (n - 1) * stride + length)
        d = to_dev(data, dev)[base_off:]
        got = as_u32(rea.crc32_batch(d, stride=stride, length=length, count=n))
        want = _oracle.crc32_uniform(data[base_off:], stride, length, n, threads=8)
        assert np.array_equal(got, want), (stride, length, n, base_off)


def test_long_packets_random_layouts(dev):
    # 60 random uniform layouts through the default path for long packets (the
    # wave-per-packet kernel from 4 KiB, the 8-packets-per-wave DMA kernel below it):
    # lengths 1.5-70 KB, strides >= length (4-B multiples: the aligned path), base offsets
    # 0-1020, counts 1-300.
    rng = np.random.default_rng(2026)
    for case in range(60):
        length = int(rng.integers(1500, 70_000))
        stride = length + 4 * int(rng.integers(0, 64)) if case % 3 else length
        stride = (stride + 3) & ~3
        base_off = 4 * int(rng.integers(0, 256))
        n = int(rng.integers(1, 300))
        data = splitmix64_bytes(case + 1, base_off + (n - 1) * stride + length)
        d = to_dev(data, dev)[base_off:]
        got = as_u32(rea.crc32_batch(d, stride=stride, length=length, count=n))
        want = _oracle.crc32_uniform(data[base_off:], stride, length, n, threads=8)
        assert np.array_equal(got, want), (case, stride, length, n, base_off)
