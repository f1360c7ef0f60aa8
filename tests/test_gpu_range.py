"""GPU parity of the batched range coder: compressed bytes, sizes
and decompressed bytes from the gfx950 kernels (through include/enet_range_amd.h) are
identical to the oracle restatement of src/c/compress.rs on the same inputs.
Run on an MI355X with  python -m pytest tests -m gpu.
"""
import json
import os

import numpy as np
import pytest

import _range_oracle as ro
from _data import ENET_SEED, enet_like_bytes, packed_offsets, ragged_lengths, splitmix64_bytes

torch = pytest.importorskip("torch")
import rusty_enet_amd as rea  # noqa: E402

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(scope="module")
def dev():
    assert torch.cuda.is_available(), "GPU tests need a HIP device"
    return torch.device("cuda:0")


def to_dev(a, dev):
    return torch.from_numpy(np.ascontiguousarray(a)).to(dev)


def windows(out: np.ndarray, offsets: np.ndarray, sizes: np.ndarray):
    return [out[int(o):int(o) + int(s)].tobytes() for o, s in zip(offsets, sizes)]


def gpu_compress(data, offs, lens, limits, dev, workers=None):
    out, out_off, sizes = rea.compress_batch(to_dev(data, dev), to_dev(offs.astype(np.int64), dev),
                                             to_dev(lens.astype(np.int32), dev),
                                             out_limits=to_dev(limits.astype(np.int32), dev), workers=workers)
    torch.cuda.synchronize()
    return out.cpu().numpy(), out_off.cpu().numpy(), sizes.cpu().numpy().astype(np.uint32)


def gpu_decompress(data, offs, lens, limits, dev, workers=None):
    out, out_off, sizes = rea.decompress_batch(to_dev(data, dev), to_dev(offs.astype(np.int64), dev),
                                               to_dev(lens.astype(np.int32), dev),
                                               to_dev(limits.astype(np.int32), dev), workers=workers)
    torch.cuda.synchronize()
    return out.cpu().numpy(), out_off.cpu().numpy(), sizes.cpu().numpy().astype(np.uint32)


def check_batch(data, lens, dev, limits=None, workers=None):
    """GPU compress vs oracle, then GPU decompress of the GPU output vs oracle and input."""
    offs = packed_offsets(lens)
    limits = lens.copy() if limits is None else limits
    g_out, g_off, g_sizes = gpu_compress(data, offs, lens, limits, dev, workers)
    o_out, o_sizes = ro.compress_ragged(data, offs, lens, packed_offsets(limits), limits)
    np.testing.assert_array_equal(g_sizes, o_sizes)
    assert windows(g_out, g_off, g_sizes) == windows(o_out, packed_offsets(limits), o_sizes)
    # decompress what the GPU produced (skip packets that did not compress)
    keep = np.nonzero(g_sizes)[0]
    if keep.size == 0:
        return g_sizes
    comp = [g_out[int(g_off[p]):int(g_off[p]) + int(g_sizes[p])] for p in keep]
    c_lens = g_sizes[keep].astype(np.uint32)
    c_data = np.concatenate(comp) if comp else np.zeros(1, np.uint8)
    c_offs = packed_offsets(c_lens)
    d_lim = np.maximum(lens[keep], 4096).astype(np.uint32)
    d_out, d_off, d_sizes = gpu_decompress(c_data, c_offs, c_lens, d_lim, dev, workers)
    od_out, od_sizes = ro.decompress_ragged(c_data, c_offs, c_lens, packed_offsets(d_lim), d_lim)
    np.testing.assert_array_equal(d_sizes, od_sizes)
    assert windows(d_out, d_off, d_sizes) == windows(od_out, packed_offsets(d_lim), od_sizes)
    src_off = packed_offsets(lens)
    for j, p in enumerate(keep):
        want = data[int(src_off[p]):int(src_off[p]) + int(lens[p])].tobytes()
        assert d_out[int(d_off[j]):int(d_off[j]) + int(d_sizes[j])].tobytes() == want, p
    return g_sizes


def test_golden_fixtures(dev):
    with open(os.path.join(HERE, "golden", "range_golden.json")) as f:
        cases = json.load(f)["cases"]
    for c in cases:
        x = rea.gather_slices([bytes.fromhex(s) for s in c["slices"]])
        lim = c["out_limit"] if c["out_limit"] is not None else 2 * len(x) + 64
        out = bytearray(lim)
        n = rea.RangeCoder().compress([bytes.fromhex(s) for s in c["slices"]], max(len(x), 1), out)
        assert bytes(out[:n]).hex() == c["compressed"], c["name"]
        if n:
            back = bytearray(8192)
            m = rea.RangeCoder().decompress(bytes(out[:n]), back)
            assert bytes(back[:m]) == x, c["name"]


def test_enet_like_ragged_batch(dev):
    lens = ragged_lengths(ENET_SEED, 3000, lo=0, hi=1392)
    data = enet_like_bytes(ENET_SEED, int(lens.sum()) + 1)
    sizes = check_batch(data, lens, dev)
    assert np.count_nonzero(sizes) > 2500  # the synthetic traffic compresses


def test_mixed_entropy_and_edge_lengths(dev):
    parts, lens = [], []
    rng = np.random.default_rng(3)
    for t in range(600):
        n = [0, 1, 2, 3, 4, 5, 63, 64, 1392, 4096][t % 10] if t < 40 else int(rng.integers(0, 1500))
        kind = t % 5
        if kind == 0:
            x = rng.integers(0, 256, n, dtype=np.uint8)
        elif kind == 1:
            x = np.zeros(n, np.uint8)
        elif kind == 2:
            x = rng.integers(0, 2, n, dtype=np.uint8)
        elif kind == 3:
            x = np.frombuffer((b"ENet command " * 400)[:n], dtype=np.uint8)
        else:
            x = enet_like_bytes(ENET_SEED + t, n)
        parts.append(x)
        lens.append(n)
    lens = np.array(lens, np.uint32)
    data = np.concatenate(parts + [np.zeros(1, np.uint8)])
    check_batch(data, lens, dev)
    # generous limits: incompressible packets code too
    check_batch(data, lens, dev, limits=(2 * lens + 64).astype(np.uint32))


def test_arena_reset_long_packets(dev):
    lens = np.array([4093, 4094, 4095, 6000, 9000, 12000], np.uint32)
    data = enet_like_bytes(ENET_SEED + 9, int(lens.sum()))
    check_batch(data, lens, dev, limits=(2 * lens).astype(np.uint32))


def test_fewer_workers_than_packets(dev):
    """Grid-stride: each lane codes many packets with one arena (state fully reset per packet)."""
    lens = ragged_lengths(ENET_SEED + 1, 1000, lo=1, hi=600)
    data = enet_like_bytes(ENET_SEED + 1, int(lens.sum()))
    for w in (3, 64, 333):
        check_batch(data, lens, dev, workers=w)


def test_tight_and_tiny_output_limits(dev):
    lens = ragged_lengths(ENET_SEED + 2, 400, lo=1, hi=800)
    data = splitmix64_bytes(ENET_SEED + 2, int(lens.sum()))  # incompressible
    sizes = check_batch(data, lens, dev)  # limit = input size: mostly 0
    assert np.count_nonzero(sizes) < 40
    check_batch(data, lens, dev, limits=np.full(lens.size, 5, np.uint32))


def test_malformed_streams(dev):
    """Arbitrary bytes fed to the decoder: sizes (incl. 0 = drop) and bytes match the oracle."""
    lens = ragged_lengths(ENET_SEED + 3, 2000, lo=1, hi=80)
    data = splitmix64_bytes(ENET_SEED + 3, int(lens.sum()))
    offs = packed_offsets(lens)
    lim = np.full(lens.size, 4092, np.uint32)
    d_out, d_off, d_sizes = gpu_decompress(data, offs, lens, lim, dev)
    o_out, o_sizes = ro.decompress_ragged(data, offs, lens, packed_offsets(lim), lim)
    np.testing.assert_array_equal(d_sizes, o_sizes)
    assert windows(d_out, d_off, d_sizes) == windows(o_out, packed_offsets(lim), o_sizes)


def test_per_call_range_coder_trait(dev):
    """RangeCoder.compress/decompress (compressor.rs:36-69 shape), incl. multi-slice input."""
    rc = rea.RangeCoder()
    slices = [b"\x80\x01\x00\x02", b"", enet_like_bytes(ENET_SEED, 300).tobytes()]
    out = bytearray(400)
    n = rc.compress(slices, 304, out)
    assert n and bytes(out[:n]) == ro.compress(slices, in_limit=304, out_limit=400)
    back = bytearray(4092)
    m = rc.decompress(bytes(out[:n]), back)
    assert bytes(back[:m]) == rea.gather_slices(slices)
    assert rc.compress([], 10, out) == 0 and rc.compress([b"abc"], 0, out) == 0
    assert rc.decompress(b"", back) == 0
