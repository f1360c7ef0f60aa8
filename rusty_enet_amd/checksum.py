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


class Context:
    """Owns an ``enet_crc_ctx`` (stream + pinned/device staging) on one device.

    Calling the context is the per-call checksum hook: ``ctx([b"..", b".."])``.
    """

    def __init__(self, device: int = 0):
        self.device = device
        handle = ctypes.c_void_p()
        check(lib().enet_crc_ctx_create(device, ctypes.byref(handle)), "enet_crc_ctx_create")
        self._handle = handle

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


_default: dict[int, Context] = {}
_default_lock = threading.Lock()


def default_context(device: int = 0) -> Context:
    with _default_lock:
        ctx = _default.get(device)
        if ctx is None:
            ctx = Context(device)
            _default[device] = ctx
        return ctx


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

    if not data.is_cuda or data.dtype != torch.uint8:
        raise ValueError("data must be a uint8 CUDA/HIP tensor")
    if stream is None:
        stream = torch.cuda.current_stream(data.device)
    sptr = stream.cuda_stream
    if offsets is not None:
        if lengths is None:
            raise ValueError("ragged batch needs offsets and lengths")
        if offsets.dtype not in (torch.int64, torch.uint64) or lengths.dtype not in (torch.int32, torch.uint32):
            raise ValueError("offsets must be 64-bit, lengths 32-bit")
        n = offsets.numel()
        if out is None:
            out = torch.empty(n, dtype=torch.int32, device=data.device)
        crc32_ragged_device(data.data_ptr(), offsets.data_ptr(), lengths.data_ptr(), n, out.data_ptr(), sptr)
        return out
    if stride is None or length is None:
        raise ValueError("uniform batch needs stride and length")
    if count is None:
        count = (data.numel() - length) // stride + 1 if data.numel() >= length else 0
    if count and (count - 1) * stride + length > data.numel():
        raise ValueError("batch extends past the end of data")
    if out is None:
        out = torch.empty(count, dtype=torch.int32, device=data.device)
    crc32_uniform_device(data.data_ptr(), stride, length, count, out.data_ptr(), sptr)
    return out


# checksum slot (SURVEY.md §8(b) batching semantics, §8(f)1-2) ------------------

def slot_adjust(crc: int, old_slot: int, new_slot: int, bytes_after_slot: int) -> int:
    """Checksum of the same datagram after its 4-byte slot changes old -> new.

    Host-side O(log n) correction (``enet_crc32_slot_adjust``); it transforms a GPU
    checksum, it never computes one.
    """
    return lib().enet_crc32_slot_adjust(crc & 0xFFFFFFFF, old_slot & 0xFFFFFFFF, new_slot & 0xFFFFFFFF,
                                        int(bytes_after_slot))


def _slot_batch_args(data, offsets, lengths, slot_offsets, slot_values):
    import torch

    if not data.is_cuda or data.dtype != torch.uint8:
        raise ValueError("data must be a uint8 CUDA/HIP tensor")
    n = offsets.numel()
    if offsets.dtype not in (torch.int64, torch.uint64):
        raise ValueError("offsets must be 64-bit")
    for name, t in (("lengths", lengths), ("slot_offsets", slot_offsets), ("slot_values", slot_values)):
        if t.dtype not in (torch.int32, torch.uint32) or t.numel() != n or not t.is_cuda:
            raise ValueError(f"{name} must be a 32-bit device tensor with one entry per datagram")
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
