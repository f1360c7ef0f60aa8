"""The C-ABI library loads, exports every symbol include/*.h declare,
and fails loudly (negative status, no CPU fallback) when no HIP device exists.
No compute calls are made here."""
import ctypes
import re

import pytest

from rusty_enet_amd import _native


def _declared_symbols():
    text = ""
    for path in _native.HEADER_PATHS:
        with open(path) as f:
            text += f.read()
    return sorted(set(re.findall(r"ENET_CRC_API\s+[\w\s\*]+?\b(enet_\w*)\s*\(", text)))


def test_header_declares_expected_api():
    syms = _declared_symbols()
    assert "enet_crc32_iov" in syms and "enet_crc32_uniform_device" in syms
    assert "enet_crc32_ragged_device" in syms and "enet_crc32_ragged_host" in syms
    assert "enet_crc32_verify_ragged_device" in syms and "enet_crc32_insert_ragged_device" in syms
    assert "enet_crc32_slot_adjust" in syms
    assert {"enet_crc_ring_create", "enet_crc_ring_submit", "enet_crc_ring_wait"} <= set(syms)
    assert {"enet_range_compress_ragged_device", "enet_range_decompress_ragged_device",
            "enet_range_scratch_bytes"} <= set(syms)
    assert {"enet_crc_ctx_create_multi", "enet_crc_ctx_lanes", "enet_crc_shard_bounds", "enet_crc32_shards_device",
            "enet_crc_ctx_set_percall_mode", "enet_crc_ctx_percall_mode", "enet_crc_ctx_stop_server"} <= set(syms)
    assert {"enet_range_compress_iov", "enet_range_decompress", "enet_range_compress_ragged_host",
            "enet_range_decompress_ragged_host"} <= set(syms)
    assert sorted(_native.exported_symbols()) == syms


def test_library_exports_every_declared_symbol():
    lib = _native.lib()
    for name in _declared_symbols():
        assert hasattr(lib, name), name
    assert lib.enet_crc_abi_version() == _native.ABI_VERSION == 6
    assert lib.enet_crc_strerror(0) == b"ok"
    assert lib.enet_crc_strerror(_native.ENET_CRC_E_NO_DEVICE) == b"no usable HIP device"


def test_only_abi_symbols_are_exported():
    import subprocess
    out = subprocess.run(["nm", "-D", "--defined-only", _native.LIB_PATH], capture_output=True, text=True).stdout
    names = {l.split()[-1] for l in out.splitlines() if l.strip()}
    ours = {n for n in names if n.startswith("enet_")}
    assert ours == set(_declared_symbols())


def test_no_device_fails_loudly():
    lib = _native.lib()
    n = lib.enet_crc_device_count()
    if n > 0:
        pytest.skip("a HIP device is visible; the no-device path is exercised on CPU-only hosts")
    handle = ctypes.c_void_p()
    st = lib.enet_crc_ctx_create(0, ctypes.byref(handle))
    assert st == _native.ENET_CRC_E_NO_DEVICE
    assert not handle.value
    import rusty_enet_amd
    with pytest.raises(rusty_enet_amd.CrcError):
        rusty_enet_amd.crc32([b"123456789"])
    # device entry points validate arguments before touching the device
    assert lib.enet_crc32_uniform_device(None, 0, 0, 0, None, None) == 0  # empty batch is a no-op
    assert lib.enet_crc32_ragged_device(None, None, None, 5, None, None) == _native.ENET_CRC_E_INVALID
    assert lib.enet_crc32_verify_ragged_device(None, None, None, None, None, 5, None, None, None) == \
        _native.ENET_CRC_E_INVALID
    assert lib.enet_crc32_insert_ragged_device(None, None, None, None, None, 0, None, None) == 0
    ring = ctypes.c_void_p()
    assert lib.enet_crc_ring_create(0, 2, 4096, 16, ctypes.byref(ring)) == _native.ENET_CRC_E_NO_DEVICE
    assert not ring.value
    assert lib.enet_crc_ring_create(0, 0, 4096, 16, ctypes.byref(ring)) == _native.ENET_CRC_E_INVALID
    assert lib.enet_crc_ring_submit(None, 0, 1) == _native.ENET_CRC_E_INVALID
    # range coder: argument checks before any device work
    assert lib.enet_range_scratch_bytes(3) == 3 * 65536
    args = [None] * 3 + [0] + [None] * 5 + [0, None]
    assert lib.enet_range_compress_ragged_device(*args) == 0  # empty batch is a no-op
    args[3] = 4
    assert lib.enet_range_compress_ragged_device(*args) == _native.ENET_CRC_E_INVALID
    assert lib.enet_range_decompress_ragged_device(*args) == _native.ENET_CRC_E_INVALID
    # multi-device context: argument checks, then the device check
    devs = (ctypes.c_int * 2)(0, 0)
    assert lib.enet_crc_ctx_create_multi(devs, 0, ctypes.byref(handle)) == _native.ENET_CRC_E_INVALID
    assert lib.enet_crc_ctx_create_multi(None, 2, ctypes.byref(handle)) == _native.ENET_CRC_E_INVALID
    assert lib.enet_crc_ctx_create_multi(devs, 2, ctypes.byref(handle)) == _native.ENET_CRC_E_NO_DEVICE
    assert not handle.value
    assert lib.enet_crc_ctx_lanes(None) == _native.ENET_CRC_E_INVALID
    assert lib.enet_crc_ctx_set_percall_mode(None, 1) == _native.ENET_CRC_E_INVALID
    assert lib.enet_crc32_shards_device(None, 0) == 0
    assert lib.enet_crc32_shards_device(None, 1) == _native.ENET_CRC_E_INVALID
    size = ctypes.c_size_t()
    assert lib.enet_range_compress_iov(None, None, 0, 1, None, 0, ctypes.byref(size)) == _native.ENET_CRC_E_INVALID
    assert lib.enet_range_decompress(None, None, 0, None, 0, ctypes.byref(size)) == _native.ENET_CRC_E_INVALID
    assert lib.enet_range_compress_ragged_host(None, *([None] * 3), 0, *([None] * 4)) == _native.ENET_CRC_E_INVALID


def test_native_shard_bounds_match_python_split():
    """enet_crc_shard_bounds (C++) == rusty_enet_amd.shards.shard_bounds (no device work)."""
    import numpy as np

    from _data import ENET_SEED, ragged_lengths
    from rusty_enet_amd.checksum import shard_bounds_native
    from rusty_enet_amd.shards import shard_bounds

    cases = [ragged_lengths(ENET_SEED, 100_000), ragged_lengths(7, 13, lo=0, hi=5000),
             np.array([], dtype=np.uint32), np.array([1000], dtype=np.uint32), np.zeros(10, dtype=np.uint32),
             np.array([0, 0, 7, 0, 0, 0, 9], dtype=np.uint32), np.full(17, 0xFFFFFFFF, dtype=np.uint32)]
    for ln in cases:
        for world in (1, 2, 3, 4, 7, 8, 64):
            got = shard_bounds_native(lengths=ln, nshards=world)
            want = [shard_bounds(world, r, lengths=ln) for r in range(world)]
            assert [(int(got[r]), int(got[r + 1])) for r in range(world)] == want, (ln.size, world)
    for count in (0, 1, 7, 1 << 20, (1 << 20) + 5):
        for world in (1, 2, 3, 8):
            got = shard_bounds_native(count=count, nshards=world)
            assert [(int(got[r]), int(got[r + 1])) for r in range(world)] == \
                [shard_bounds(world, r, count=count) for r in range(world)]
