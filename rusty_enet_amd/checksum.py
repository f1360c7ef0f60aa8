"""Host-side mirror of rusty_enet's checksum surface, backed by the gfx950 kernels.

Reference interface (jabuwu/rusty_enet v0.4.0):
  * ``pub fn crc32(in_buffers: &[&[u8]]) -> u32``               src/crc32.rs:39-47
  * ``HostSettings::checksum: Option<Box<dyn Fn(&[&[u8]]) -> u32>>`` src/host.rs:40
    (installed as ``Some(Box::new(enet::crc32))`` in examples/server.rs:17)

``crc32(in_buffers)`` here takes the same argument (a sequence of byte slices,
checksummed as their concatenation) and returns the same u32.  Unlike the
reference it can fail: without the native library or a HIP device it raises
(NativeLibraryMissing / CrcError) instead of silently computing on the CPU.

Batch entry points (one kernel launch for many packets) are what the GPU is
for; the per-call path pays a launch + two PCIe copies per datagram.
"""
from __future__ import annotations

import atexit
import ctypes
import threading
from typing import Iterable, Optional, Sequence

import numpy as np

from . import _native
from ._native import Iov, check, lib

BytesLike = "bytes | bytearray | memoryview | np.ndarray"


def _as_u8(buf) -> np.ndarray:
    if isinstance(buf, np.ndarray):
        a = buf.reshape(-1).view(np.uint8) if buf.dtype != np.uint8 else buf.reshape(-1)
        return np.ascontiguousarray(a)
    return np.frombuffer(buf, dtype=np.uint8)


def _writable_u8(buf) -> np.ndarray:
    """A writable uint8 view of ``buf`` (bytearray, memoryview, numpy array) without a copy."""
    if isinstance(buf, np.ndarray):
        if not buf.flags.c_contiguous or not buf.flags.writeable:
            raise ValueError("out must be a writable contiguous array")
        return buf.reshape(-1).view(np.uint8)
    a = np.frombuffer(memoryview(buf).cast("B"), dtype=np.uint8)
    if not a.flags.writeable:
        raise ValueError("out must be writable")
    return a


def shard_bounds_native(lengths=None, count: Optional[int] = None, nshards: int = 1) -> np.ndarray:
    """``enet_crc_shard_bounds``: the C++ byte-balanced split (nshards + 1 bounds)."""
    if lengths is not None:
        ln = np.ascontiguousarray(lengths, dtype=np.uint32)
        count = ln.size
        ptr = ln.ctypes.data if ln.size else None
    else:
        ln, ptr = None, None
    bounds = np.zeros(nshards + 1, dtype=np.uint64)
    check(lib().enet_crc_shard_bounds(ptr, int(count or 0), nshards, bounds.ctypes.data), "enet_crc_shard_bounds")
    return bounds


class Context:
    """Owns an ``enet_crc_ctx`` (streams + pinned/device staging) on one device, or on a
    device list (``devices=[0, 1, ...]``, duplicates allowed): host-memory batches are
    then split into byte-balanced shards checksummed on all lanes at once.

    Calling the context is the per-call checksum hook: ``ctx([b"..", b".."])``.
    """

    def __init__(self, device: int = 0, devices: Optional[Sequence[int]] = None):
        devs = [int(d) for d in (devices if devices is not None else [device])]
        if not devs:
            raise ValueError("empty device list")
        self.device = devs[0]
        self.devices = devs
        handle = ctypes.c_void_p()
        arr = (ctypes.c_int * len(devs))(*devs)
        check(lib().enet_crc_ctx_create_multi(arr, len(devs), ctypes.byref(handle)), "enet_crc_ctx_create_multi")
        self._handle = handle

    @property
    def lanes(self) -> int:
        return lib().enet_crc_ctx_lanes(self._handle)

    def set_percall_mode(self, mode: int) -> None:
        """``_native.ENET_CRC_PERCALL_COPY``, ``ENET_CRC_PERCALL_ZEROCOPY`` (the default: one
        launch per call, nothing resident) or ``ENET_CRC_PERCALL_PERSISTENT`` (opt-in: a
        resident server wave; include/enet_crc_amd.h has what it holds while it runs)."""
        check(lib().enet_crc_ctx_set_percall_mode(self._handle, mode), "enet_crc_ctx_set_percall_mode")

    @property
    def percall_mode(self) -> int:
        mode = lib().enet_crc_ctx_percall_mode(self._handle)
        if mode < 0:
            check(mode, "enet_crc_ctx_percall_mode")
        return mode

    def stop_server(self) -> None:
        """Stop the persistent server wave now, if one runs (e.g. before a device-wide
        synchronisation, which would otherwise wait up to its 20-ms idle exit)."""
        check(lib().enet_crc_ctx_stop_server(self._handle), "enet_crc_ctx_stop_server")

    @property
    def handle(self) -> int:
        return self._handle.value

    def close(self) -> None:
        if self._handle is not None and self._handle.value:
            lib().enet_crc_ctx_destroy(self._handle)
        self._handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    # src/crc32.rs:39 -------------------------------------------------------
    def crc32(self, in_buffers: Sequence) -> int:
        arrays = [_as_u8(b) for b in in_buffers]
        iovs = (Iov * max(1, len(arrays)))()
        for i, a in enumerate(arrays):
            iovs[i].data = a.ctypes.data if a.size else None
            iovs[i].len = a.size
        out = ctypes.c_uint32()
        check(lib().enet_crc32_iov(self._handle, iovs, len(arrays), ctypes.byref(out)), "enet_crc32_iov")
        return out.value

    __call__ = crc32

    # host-resident batch (end-to-end path) ---------------------------------
    def crc32_ragged_host(self, data, offsets, lengths) -> np.ndarray:
        d = _as_u8(data)
        off = np.ascontiguousarray(offsets, dtype=np.uint64)
        ln = np.ascontiguousarray(lengths, dtype=np.uint32)
        if off.shape != ln.shape:
            raise ValueError("offsets and lengths must have the same shape")
        if off.size and int((off + ln).max()) > d.size:
            raise ValueError("a packet extends past the end of data")
        out = np.empty(off.size, dtype=np.uint32)
        check(lib().enet_crc32_ragged_host(self._handle, d.ctypes.data, off.ctypes.data, ln.ctypes.data,
                                           off.size, out.ctypes.data), "enet_crc32_ragged_host")
        return out

    # range coder, host memory (src/compressor.rs:9-14) ---------------------
    def range_compress(self, in_buffers: Sequence, in_limit: int, out) -> int:
        """``Compressor::compress(in_buffers, in_limit, out)``: writes into ``out`` (a
        writable buffer), returns the reference's size (0 = not coded)."""
        arrays = [_as_u8(b) for b in in_buffers]
        iovs = (Iov * max(1, len(arrays)))()
        for i, a in enumerate(arrays):
            iovs[i].data = a.ctypes.data if a.size else None
            iovs[i].len = a.size
        dst = _writable_u8(out)
        size = ctypes.c_size_t()
        check(lib().enet_range_compress_iov(self._handle, iovs, len(arrays), int(in_limit),
                                            dst.ctypes.data if dst.size else None, dst.size, ctypes.byref(size)),
              "enet_range_compress_iov")
        return size.value

    def range_decompress(self, in_data, out) -> int:
        """``Compressor::decompress(in_data, out)``."""
        src = _as_u8(in_data)
        dst = _writable_u8(out)
        size = ctypes.c_size_t()
        check(lib().enet_range_decompress(self._handle, src.ctypes.data if src.size else None, src.size,
                                          dst.ctypes.data if dst.size else None, dst.size, ctypes.byref(size)),
              "enet_range_decompress")
        return size.value

    def range_ragged_host(self, decompress: bool, data, offsets, lengths, out_limits):
        """Batch of packets in host memory; returns (out bytes, out offsets, sizes)."""
        d = _as_u8(data)
        off = np.ascontiguousarray(offsets, dtype=np.uint64)
        ln = np.ascontiguousarray(lengths, dtype=np.uint32)
        lim = np.ascontiguousarray(out_limits, dtype=np.uint32)
        if not (off.shape == ln.shape == lim.shape):
            raise ValueError("offsets, lengths and out_limits must have the same shape")
        if off.size and int((off + ln).max()) > d.size:
            raise ValueError("a packet extends past the end of data")
        o_off = np.zeros(off.size, dtype=np.uint64)
        if off.size > 1:
            np.cumsum(lim[:-1], dtype=np.uint64, out=o_off[1:])
        out = np.zeros(max(1, int(lim.sum(dtype=np.uint64))), dtype=np.uint8)
        sizes = np.zeros(off.size, dtype=np.uint32)
        fn = lib().enet_range_decompress_ragged_host if decompress else lib().enet_range_compress_ragged_host
        check(fn(self._handle, d.ctypes.data, off.ctypes.data, ln.ctypes.data, off.size, out.ctypes.data,
                 o_off.ctypes.data, lim.ctypes.data, sizes.ctypes.data),
              "enet_range_decompress_ragged_host" if decompress else "enet_range_compress_ragged_host")
        return out, o_off, sizes


_default: dict[int, Context] = {}
_default_lock = threading.Lock()


def default_context(device: int = 0) -> Context:
    with _default_lock:
        ctx = _default.get(device)
        if ctx is None:
            if not _default:
                atexit.register(_close_defaults)
            ctx = Context(device)
            _default[device] = ctx
        return ctx


def _close_defaults() -> None:
    """At interpreter exit: stop each default context's per-call server wave (it would
    otherwise run until its 20-ms idle limit while the process tears the device down)."""
    with _default_lock:
        for ctx in _default.values():
            ctx.close()
        _default.clear()


def crc32(in_buffers: Sequence) -> int:
    """Mirror of ``rusty_enet::crc32`` (src/crc32.rs:39): CRC of the concatenation."""
    return default_context(0).crc32(in_buffers)


def checksum_fn(device: int = 0):
    """The value to store in ``HostSettings.checksum`` (src/host.rs:40)."""
    return default_context(device)


# device-resident batches (raw pointers; any framework's device memory) -------

def crc32_uniform_device(base_ptr: int, stride: int, length: int, count: int, out_ptr: int,
                         stream: Optional[int] = None) -> None:
    check(lib().enet_crc32_uniform_device(base_ptr, stride, length, count, out_ptr, stream or None),
          "enet_crc32_uniform_device")


def crc32_ragged_device(base_ptr: int, offsets_ptr: int, lengths_ptr: int, count: int, out_ptr: int,
                        stream: Optional[int] = None) -> None:
    check(lib().enet_crc32_ragged_device(base_ptr, offsets_ptr, lengths_ptr, count, out_ptr, stream or None),
          "enet_crc32_ragged_device")


def crc32_batch(data, *, offsets=None, lengths=None, stride: Optional[int] = None,
                length: Optional[int] = None, count: Optional[int] = None, out=None, stream=None):
    """Checksum a device-resident batch held in torch tensors (torch = plumbing only).

    Uniform: ``crc32_batch(data, stride=S, length=L, count=N)``.
    Ragged:  ``crc32_batch(data, offsets=off_u64, lengths=len_i32)``.
    Returns an int32 tensor whose bits are the u32 checksums (``.view(torch.uint32)``
    or ``& 0xFFFFFFFF`` in Python to read them unsigned).  Runs on ``stream`` (a
    torch.cuda.Stream) or torch's current stream.
    """
    import torch

    if not data.is_cuda or data.dtype != torch.uint8 or not data.is_contiguous():
        raise ValueError("data must be a contiguous uint8 CUDA/HIP tensor")
    dev = data.device
    if stream is None:
        stream = torch.cuda.current_stream(dev)
    elif stream.device != dev:
        raise ValueError("stream must belong to the data's device")
    sptr = stream.cuda_stream
    if offsets is not None:
        if lengths is None:
            raise ValueError("ragged batch needs offsets and lengths")
        _check_dev(dev, offsets=(offsets, (torch.int64, torch.uint64)), lengths=(lengths, (torch.int32, torch.uint32)))
        n = offsets.numel()
        if lengths.numel() != n:
            raise ValueError("offsets and lengths must have one entry per packet")
        if out is None:
            out = torch.empty(n, dtype=torch.int32, device=dev)
        _check_dev(dev, out=(out, (torch.int32, torch.uint32)))
        if out.numel() < n:
            raise ValueError("out is too small")
        with torch.cuda.device(dev):
            crc32_ragged_device(data.data_ptr(), offsets.data_ptr(), lengths.data_ptr(), n, out.data_ptr(), sptr)
        return out
    if stride is None or length is None:
        raise ValueError("uniform batch needs stride and length")
    if stride < 0 or length < 0 or length > 0xFFFFFFFF:
        raise ValueError("stride and length must be non-negative (length < 2**32)")
    if count is None:
        count = (data.numel() - length) // stride + 1 if data.numel() >= length and stride else 0
    if count < 0:
        raise ValueError("count must be non-negative")
    if count and (count - 1) * stride + length > data.numel():
        raise ValueError("batch extends past the end of data")
    if out is None:
        out = torch.empty(count, dtype=torch.int32, device=dev)
    _check_dev(dev, out=(out, (torch.int32, torch.uint32)))
    if out.numel() < count:
        raise ValueError("out is too small")
    with torch.cuda.device(dev):
        crc32_uniform_device(data.data_ptr(), stride, length, count, out.data_ptr(), sptr)
    return out


def _check_dev(dev, **tensors) -> None:
    """Every tensor on `dev`, contiguous, with one of the allowed dtypes."""
    for name, (t, dtypes) in tensors.items():
        if not t.is_cuda or t.device != dev:
            raise ValueError(f"{name} must be on {dev}")
        if t.dtype not in dtypes:
            raise ValueError(f"{name} must have dtype in {dtypes}")
        if not t.is_contiguous():
            raise ValueError(f"{name} must be contiguous")


def device_status(device: int = 0, clear: bool = False) -> int:
    """``enet_crc_device_status``: the device's failure bits (0 = none) since the last clear.

    A batch kernel that gave up on an inter-wave wait sets them (include/enet_crc_amd.h);
    after the asynchronous device entries (``crc32_batch``, ``verify_batch``, ...) a caller
    that must not trust a failed batch synchronises and checks this.  The synchronous host
    entries raise ``CrcError`` with ``ENET_CRC_E_DEVICE`` instead.
    """
    st = lib().enet_crc_device_status(int(device), 1 if clear else 0)
    if st < 0:
        check(st, "enet_crc_device_status")
    return st


def crc32_shards_device(shards: Sequence[dict]) -> None:
    """``enet_crc32_shards_device``: one batch per device, launched on every device at
    once.  Each shard is a dict with ``data`` (uint8 tensor) and either ``stride``/
    ``length``/``count`` or ``offsets``/``lengths``, plus ``out`` (int32 tensor) and an
    optional ``stream`` (torch stream of that device)."""
    import torch

    arr = (_native.Shard * max(1, len(shards)))()
    for i, sh in enumerate(shards):
        data, out = sh["data"], sh["out"]
        dev = data.device
        if not data.is_cuda or data.dtype != torch.uint8:
            raise ValueError("data must be a uint8 device tensor")
        _check_dev(dev, out=(out, (torch.int32, torch.uint32)))
        stream = sh.get("stream") or torch.cuda.current_stream(dev)
        arr[i].device = dev.index
        arr[i].d_base = data.data_ptr()
        arr[i].d_out = out.data_ptr()
        arr[i].hip_stream = stream.cuda_stream
        if "offsets" in sh:
            off, ln = sh["offsets"], sh["lengths"]
            _check_dev(dev, offsets=(off, (torch.int64, torch.uint64)), lengths=(ln, (torch.int32, torch.uint32)))
            arr[i].d_offsets, arr[i].d_lengths, arr[i].count = off.data_ptr(), ln.data_ptr(), off.numel()
        else:
            arr[i].stride, arr[i].length, arr[i].count = sh["stride"], sh["length"], sh["count"]
            if arr[i].count and (arr[i].count - 1) * arr[i].stride + arr[i].length > data.numel():
                raise ValueError("shard extends past the end of its data")
        if out.numel() < arr[i].count:
            raise ValueError("out is too small")
    check(lib().enet_crc32_shards_device(arr, len(shards)), "enet_crc32_shards_device")


# checksum slot (SURVEY.md §8(b) batching semantics, §8(f)1-2) ------------------

def slot_adjust(crc: int, old_slot: int, new_slot: int, bytes_after_slot: int) -> int:
    """Checksum of the same datagram after its 4-byte slot changes old -> new.

    Host-side O(log n) correction (``enet_crc32_slot_adjust``); it transforms a GPU
    checksum, it never computes one.
    """
    return lib().enet_crc32_slot_adjust(crc & 0xFFFFFFFF, old_slot & 0xFFFFFFFF, new_slot & 0xFFFFFFFF,
                                        int(bytes_after_slot))


def crc32_combine(crc_a: int, crc_b: int, len_b: int) -> int:
    """``crc32(&[a, b])`` from ``crc32(&[a])``, ``crc32(&[b])`` and ``len(b)``.

    Host-side merge (``enet_crc32_combine``): the merged digest of shards checksummed
    on different GPUs, without touching the bytes again.
    """
    if len_b < 0:
        raise ValueError("len_b must be >= 0")
    return lib().enet_crc32_combine(crc_a & 0xFFFFFFFF, crc_b & 0xFFFFFFFF, int(len_b))


def _slot_batch_args(data, offsets, lengths, slot_offsets, slot_values):
    import torch

    if not data.is_cuda or data.dtype != torch.uint8 or not data.is_contiguous():
        raise ValueError("data must be a contiguous uint8 CUDA/HIP tensor")
    n = offsets.numel()
    i32 = (torch.int32, torch.uint32)
    _check_dev(data.device, offsets=(offsets, (torch.int64, torch.uint64)), lengths=(lengths, i32),
               slot_offsets=(slot_offsets, i32), slot_values=(slot_values, i32))
    for name, t in (("lengths", lengths), ("slot_offsets", slot_offsets), ("slot_values", slot_values)):
        if t.numel() != n:
            raise ValueError(f"{name} must have one entry per datagram")
    return n


def verify_batch(data, offsets, lengths, slot_offsets, slot_values, stream=None):
    """Batched receive verify (src/c/protocol.rs:1470-1502 per datagram), device tensors.

    Returns ``(crc, ok)`` int32 tensors: ``crc[p]`` is the checksum the reference
    computes at :1499 (slot := slot_values[p]), ``ok[p]`` 1 to accept, 0 to drop.
    ``data`` is not modified.
    """
    import torch

    n = _slot_batch_args(data, offsets, lengths, slot_offsets, slot_values)
    stream = stream or torch.cuda.current_stream(data.device)
    crc = torch.empty(n, dtype=torch.int32, device=data.device)
    ok = torch.empty(n, dtype=torch.int32, device=data.device)
    check(lib().enet_crc32_verify_ragged_device(data.data_ptr(), offsets.data_ptr(), lengths.data_ptr(),
                                                slot_offsets.data_ptr(), slot_values.data_ptr(), n,
                                                crc.data_ptr(), ok.data_ptr(), stream.cuda_stream),
          "enet_crc32_verify_ragged_device")
    return crc, ok


def insert_batch(data, offsets, lengths, slot_offsets, slot_values, stream=None):
    """Batched send insert (src/c/protocol.rs:2255-2293), in place on device tensors.

    Each datagram's slot takes slot_values[p], the datagram is checksummed and the
    checksum is written into the slot (native-endian).  Returns the checksums.
    """
    import torch

    n = _slot_batch_args(data, offsets, lengths, slot_offsets, slot_values)
    stream = stream or torch.cuda.current_stream(data.device)
    crc = torch.empty(n, dtype=torch.int32, device=data.device)
    check(lib().enet_crc32_insert_ragged_device(data.data_ptr(), offsets.data_ptr(), lengths.data_ptr(),
                                                slot_offsets.data_ptr(), slot_values.data_ptr(), n,
                                                crc.data_ptr(), stream.cuda_stream),
          "enet_crc32_insert_ragged_device")
    return crc
