"""GPU tests of the multi-device context, the sharded device entry point, the per-call
modes, the error path of the host pipeline and the host-memory range-coder entry
points -- all through the C ABI, bit-exact against the oracles.

On the 1-GPU box a device list [0, 0] gives two lanes (two shards, two worker
threads, two stream pairs) on the one device: the same code path as [0, 1, ..., 7]
on an 8-GPU node, where each lane sits on its own device.
"""
import ctypes
import os

import numpy as np
import pytest

import _oracle
import _range_oracle as ro
from _data import ENET_SEED, enet_like_bytes, packed_offsets, ragged_lengths, splitmix64_bytes

torch = pytest.importorskip("torch")
import rusty_enet_amd as rea  # noqa: E402
from rusty_enet_amd import _native  # noqa: E402
from rusty_enet_amd.protocol import (HEADER_FLAG_COMPRESSED, PROTOCOL_MAXIMUM_PEER_ID,  # noqa: E402
                                     verify_received)

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    assert torch.cuda.is_available(), "GPU tests need a HIP device"
    return torch.device("cuda:0")


def test_two_lanes_on_one_device_bit_exact(dev):
    lengths = ragged_lengths(21, 300_000, lo=0, hi=1392)
    offsets = packed_offsets(lengths) + np.uint64(3)
    data = splitmix64_bytes(22, int(lengths.sum()) + 8)
    want = _oracle.crc32_ragged(data, offsets, lengths)
    with rea.Context(devices=[0, 0]) as ctx:
        assert ctx.lanes == 2
        assert np.array_equal(ctx.crc32_ragged_host(data, offsets, lengths), want)
        # more lanes than packets, and a batch whose shards cross the 256K-packet chunking
        assert np.array_equal(ctx.crc32_ragged_host(data, offsets[:1], lengths[:1]), want[:1])
    with rea.Context(devices=[0, 0, 0, 0]) as ctx:
        assert ctx.lanes == 4
        assert np.array_equal(ctx.crc32_ragged_host(data, offsets[:3], lengths[:3]), want[:3])
        assert np.array_equal(ctx.crc32_ragged_host(data, offsets, lengths), want)
        assert ctx.crc32([data[:1392]]) == _oracle.crc32([data[:1392]])  # per-call path: lane 0


def test_full_shard_sizes_through_a_two_lane_context(dev):
    # 2 lanes x 600K packets of up to 1392 B: each lane pipelines several chunks.
    lengths = ragged_lengths(23, 1_200_000)
    offsets = packed_offsets(lengths)
    data = splitmix64_bytes(24, int(lengths.sum()))
    with rea.Context(devices=[0, 0]) as ctx:
        got = ctx.crc32_ragged_host(data, offsets, lengths)
    assert np.array_equal(got, _oracle.crc32_ragged(data, offsets, lengths))


def test_shards_device_two_shards(dev):
    n, L = 50_000, 1200
    a = splitmix64_bytes(27, n * L)
    lengths = ragged_lengths(28, 40_000, lo=0, hi=4096)
    offsets = packed_offsets(lengths) + np.uint64(1)
    b = splitmix64_bytes(29, int(lengths.sum()) + 8)
    da, db = torch.from_numpy(a).to(dev), torch.from_numpy(b).to(dev)
    oa = torch.empty(n, dtype=torch.int32, device=dev)
    ob = torch.empty(lengths.size, dtype=torch.int32, device=dev)
    s2 = torch.cuda.Stream(device=dev)
    # A third shard of 64-KiB buffers (the wave-per-packet kernel) on a stream of its own.
    nc, LC = 96, 65536
    cb = splitmix64_bytes(30, nc * LC)
    dc = torch.from_numpy(cb).to(dev)
    oc = torch.empty(nc, dtype=torch.int32, device=dev)
    s3 = torch.cuda.Stream(device=dev)
    rea.crc32_shards_device([
        {"data": da, "stride": L, "length": L, "count": n, "out": oa},
        {"data": db, "offsets": torch.from_numpy(offsets.astype(np.int64)).to(dev),
         "lengths": torch.from_numpy(lengths.astype(np.int32)).to(dev), "out": ob, "stream": s2},
        {"data": dc, "stride": LC, "length": LC, "count": nc, "out": oc, "stream": s3},
    ])
    torch.cuda.synchronize()
    assert np.array_equal(oc.cpu().numpy().view(np.uint32), _oracle.crc32_uniform(cb, LC, LC, nc, threads=8))
    assert np.array_equal(oa.cpu().numpy().view(np.uint32), _oracle.crc32_uniform(a, L, L, n, threads=8))
    assert np.array_equal(ob.cpu().numpy().view(np.uint32), _oracle.crc32_ragged(b, offsets, lengths))
    # Merged digest of shard a: its packets are back to back, so the
    # GPU's per-packet checksums fold (enet_crc32_combine) into the checksum of its bytes.
    digest = None
    for c in oa.cpu().numpy().view(np.uint32).tolist():
        digest = c if digest is None else rea.crc32_combine(digest, c, L)
    assert digest == _oracle.crc32([a])


def test_shards_device_rejects_misplaced_shards(dev):
    """enet_crc32_shards_device checks every shard's placement before
    anything launches.  A shard naming another device than the one its buffers live on
    (E_INVALID; on a 1-GPU box the index itself is bad: E_NO_DEVICE), a shard whose input
    or output is host memory, or whose stream belongs to another device, fails the whole
    call, and the valid shard in front of it does not run."""
    n, L = 4096, 1200
    a = torch.from_numpy(splitmix64_bytes(51, n * L)).to(dev)
    oa = torch.full((n,), 7, dtype=torch.int32, device=dev)
    ob = torch.full((n,), 7, dtype=torch.int32, device=dev)
    host_out = torch.zeros(n, dtype=torch.int32).pin_memory()
    stream = torch.cuda.current_stream(dev).cuda_stream

    def shard(device, base, out, s=stream):
        sh = _native.Shard()
        sh.device, sh.d_base, sh.d_offsets, sh.d_lengths = device, base, None, None
        sh.stride, sh.length, sh.count, sh.d_out, sh.hip_stream = L, L, n, out, s
        return sh

    lib = _native.lib()
    ndev = torch.cuda.device_count()
    bad_dev_status = _native.ENET_CRC_E_INVALID if ndev > 1 else _native.ENET_CRC_E_NO_DEVICE
    cases = [
        (shard(1, a.data_ptr(), ob.data_ptr()), bad_dev_status),           # pointers on device 0
        (shard(0, a.data_ptr(), host_out.data_ptr()), _native.ENET_CRC_E_INVALID),  # output in host memory
        (shard(0, host_out.data_ptr(), ob.data_ptr()), _native.ENET_CRC_E_INVALID),  # input in host memory
        (shard(-1, a.data_ptr(), ob.data_ptr()), _native.ENET_CRC_E_NO_DEVICE),
    ]
    if ndev > 1:
        s1 = torch.cuda.Stream(device=torch.device("cuda", 1))
        cases.append((shard(0, a.data_ptr(), ob.data_ptr(), s1.cuda_stream), _native.ENET_CRC_E_INVALID))
    for bad, status in cases:
        arr = (_native.Shard * 2)(shard(0, a.data_ptr(), oa.data_ptr()), bad)
        assert lib.enet_crc32_shards_device(arr, 2) == status
        torch.cuda.synchronize()
        assert bool((oa == 7).all()) and bool((ob == 7).all())  # nothing launched
    arr = (_native.Shard * 1)(shard(0, a.data_ptr(), oa.data_ptr()))
    assert lib.enet_crc32_shards_device(arr, 1) == 0
    torch.cuda.synchronize()
    assert np.array_equal(oa.cpu().numpy().view(np.uint32), _oracle.crc32_uniform(a.cpu().numpy(), L, L, n))


@pytest.mark.parametrize("mode", [_native.ENET_CRC_PERCALL_COPY, _native.ENET_CRC_PERCALL_ZEROCOPY,
                                  _native.ENET_CRC_PERCALL_PERSISTENT])
def test_per_call_modes(dev, mode):
    with rea.Context(0) as ctx:
        ctx.set_percall_mode(mode)
        assert ctx([bytes([1, 2, 3, 4, 5, 6, 7, 8])]) == 3314076223                        # src/crc32.rs:52
        assert ctx([bytes([1, 2, 3, 4, 5, 6, 7, 8]), bytes([8, 7, 6, 5, 4, 3, 2, 1])]) == 1712484799
        assert ctx([]) == 0 and ctx([b""]) == 0
        for n in (1, 3, 4, 5, 17, 1200, 1392, 1396, 4095, 4096, 65536, 100_003):
            buf = splitmix64_bytes(n, n)
            assert ctx([buf]) == _oracle.crc32([buf]), n
        rng = np.random.default_rng(3)
        for trial in range(10):
            slices = [splitmix64_bytes(100 * trial + j, int(rng.integers(0, 40)) if j < 9 else 0) for j in range(65)]
            assert ctx(slices) == _oracle.crc32(slices)


def test_persistent_server_lifecycle(dev):
    """ENET_CRC_PERCALL_PERSISTENT: every length a datagram can have (0..4096, the
    mailbox window) bit-exact, across the server's idle exit and relaunch, a switch to
    another mode and back, and destroying the context while the server runs."""
    import time
    rng = np.random.default_rng(11)
    with rea.Context(0) as ctx:
        ctx.set_percall_mode(_native.ENET_CRC_PERCALL_PERSISTENT)
        for n in list(range(0, 130)) + [int(x) for x in rng.integers(130, 4097, 300)] + [4096]:
            buf = splitmix64_bytes(7 * n + 1, n)
            cut = int(rng.integers(0, n + 1))
            assert ctx([buf[:cut], buf[cut:]]) == _oracle.crc32([buf]), n
        time.sleep(0.1)  # > 20 ms idle: the server has exited; the next call relaunches it
        assert ctx([bytes([1, 2, 3, 4, 5, 6, 7, 8])]) == 3314076223
        ctx.set_percall_mode(_native.ENET_CRC_PERCALL_ZEROCOPY)  # stops the server
        assert ctx([b"abc"]) == _oracle.crc32([b"abc"])
        ctx.set_percall_mode(_native.ENET_CRC_PERCALL_PERSISTENT)
        assert ctx([b"abc"]) == _oracle.crc32([b"abc"])
    # the context was destroyed with the server running; a new one starts its own
    with rea.Context(0) as ctx:
        ctx.set_percall_mode(_native.ENET_CRC_PERCALL_PERSISTENT)
        assert ctx([b"123456789"]) == _oracle.crc32([b"123456789"])


def test_stream_device_is_used(dev):
    """The device entry points launch on the stream's device; on one GPU this
    checks that an explicit stream of device 0 works whatever the current device is."""
    n, L = 4096, 1200
    data = splitmix64_bytes(30, n * L)
    d = torch.from_numpy(data).to(dev)
    s = torch.cuda.Stream(device=dev)
    out = rea.crc32_batch(d, stride=L, length=L, count=n, stream=s)
    s.synchronize()
    assert np.array_equal(out.cpu().numpy().view(np.uint32), _oracle.crc32_uniform(data, L, L, n))
    with pytest.raises(ValueError):
        rea.crc32_batch(d, stride=L, length=L, count=n + 1)
    with pytest.raises(ValueError):
        rea.crc32_batch(d, offsets=torch.zeros(3, dtype=torch.int64), lengths=torch.ones(3, dtype=torch.int32,
                                                                                         device=dev))


# --- range coder, host-memory entry points (src/compressor.rs:9-14) ----------------------

def test_range_compress_iov_matches_oracle(dev):
    with rea.Context(0) as ctx:
        rng = np.random.default_rng(5)
        for trial in range(40):
            nsl = int(rng.integers(1, 6))
            slices = [enet_like_bytes(trial * 10 + j, int(rng.integers(0, 300))).tobytes() for j in range(nsl)]
            if trial % 4 == 1 and nsl > 1:
                slices[1] = b""  # empty middle slice: one 0 byte (compress.rs:119-122)
            total = len(rea.gather_slices(slices))
            lim = int(rng.integers(1, 2 * total + 64)) if trial % 3 == 0 else 2 * total + 64
            out = bytearray(lim)
            n = ctx.range_compress(slices, max(total, 1), out)
            assert bytes(out[:n]) == ro.compress(slices, in_limit=max(total, 1), out_limit=lim), trial
            if n:
                back = bytearray(4096)
                m = ctx.range_decompress(bytes(out[:n]), back)
                assert bytes(back[:m]) == rea.gather_slices(slices)
        assert ctx.range_compress([], 10, bytearray(10)) == 0
        assert ctx.range_compress([b"abc"], 0, bytearray(10)) == 0
        assert ctx.range_decompress(b"", bytearray(10)) == 0


def test_range_ragged_host_matches_oracle(dev):
    lens = ragged_lengths(31, 5000, lo=0, hi=1392)
    data = enet_like_bytes(32, int(lens.sum()) + 1)
    offs = packed_offsets(lens)
    with rea.Context(0) as ctx:
        out, o_off, sizes = ctx.range_ragged_host(False, data, offs, lens, lens)
        w_out, w_sizes = ro.compress_ragged(data, offs, lens, packed_offsets(lens), lens)
        assert np.array_equal(sizes, w_sizes)
        for p in range(lens.size):
            a, b = int(o_off[p]), int(packed_offsets(lens)[p])
            assert out[a:a + sizes[p]].tobytes() == w_out[b:b + w_sizes[p]].tobytes(), p
        coded = np.nonzero(sizes)[0]
        c_len = sizes[coded]
        c_off = packed_offsets(c_len)
        blob = np.concatenate([out[int(o_off[p]):int(o_off[p]) + int(sizes[p])] for p in coded])
        back, b_off, b_sizes = ctx.range_ragged_host(True, blob, c_off, c_len, np.full(coded.size, 4096, np.uint32))
        assert np.array_equal(b_sizes, lens[coded])
        for j, p in enumerate(coded):
            assert back[int(b_off[j]):int(b_off[j]) + int(b_sizes[j])].tobytes() == \
                data[int(offs[p]):int(offs[p]) + int(lens[p])].tobytes()


def _compressed_datagram(peer_id: int, connect_id: int, commands: bytes, seed: int) -> bytes:
    """What the reference send path puts on the wire with a range coder and a checksum
    (protocol.rs:2213-2299): header with the COMPRESSED flag, the checksum over header +
    slot(connect_id) + UNCOMPRESSED commands, then the compressed commands."""
    raw = (peer_id | HEADER_FLAG_COMPRESSED) & 0xFFFF
    header = bytes([raw >> 8, raw & 0xFF])
    c = ro.compress([commands], in_limit=len(commands), out_limit=len(commands))
    assert 0 < len(c) < len(commands)
    slot_v = 0 if peer_id == PROTOCOL_MAXIMUM_PEER_ID else connect_id
    hdr = (ctypes.c_uint8 * 6)(*header, 0, 0, 0, 0)
    body = np.frombuffer(commands, dtype=np.uint8).copy()
    rest = (_oracle.OracleIov * 1)(_oracle.OracleIov(body.ctypes.data, body.size))
    crc = _oracle.lib().oracle_enet_insert(hdr, 2, rest, 1, slot_v)
    return header + crc.to_bytes(4, "little") + c


def test_verify_received_decompresses_before_the_checksum(dev):
    """a compressed datagram's checksum covers header + DECOMPRESSED commands
    (protocol.rs:1441-1502)."""
    cmds = [enet_like_bytes(40 + i, 200 + 37 * i).tobytes() for i in range(6)]
    grams = [_compressed_datagram(5, 0x1234567, c, i) for i, c in enumerate(cmds)]
    # a corrupted one (flip a compressed byte) and one with the wrong connect_id
    bad = bytearray(grams[2])
    bad[-3] ^= 0x40
    grams[2] = bytes(bad)
    grams.append(_compressed_datagram(6, 99, cmds[0], 9))
    ids = {5: 0x1234567, 6: 98}
    with rea.Context(0) as ctx:
        got = verify_received(grams, lambda pid: ids[pid], ctx=ctx, compressor=True)
        assert got == [True, True, False, True, True, True, False]
        # without a compressor the reference drops compressed datagrams (:1442-1444)
        assert verify_received(grams, lambda pid: ids[pid], ctx=ctx) == [False] * len(grams)
