"""Host-side mirror of rusty_enet's `Compressor` / `RangeCoder`, backed by the gfx950 kernels.

Reference interface (jabuwu/rusty_enet v0.4.0, src/compressor.rs):
  * ``trait Compressor { fn compress(&mut self, in_buffers: &[&[u8]], in_limit: usize,
    out: &mut [u8]) -> usize; fn decompress(&mut self, in_data: &[u8], out: &mut [u8]) -> usize; }``
    (:9-14)
  * ``RangeCoder::new()`` (:22-28) and its impl (:36-69) over src/c/compress.rs.

``RangeCoder.compress`` / ``.decompress`` take the same arguments and return the same
sizes (0 = not compressible within ``len(out)`` / malformed stream); they call the
host-memory C entry points ``enet_range_compress_iov`` / ``enet_range_decompress`` on a
context that owns the arenas, so they pay a launch and two PCIe copies per call.
``compress_batch`` / ``decompress_batch`` are the real interface (one launch for a
whole batch of device-resident datagrams, include/enet_range_amd.h).  There is no
CPU fallback: without the library or a device these raise.
"""
from __future__ import annotations

from typing import Optional, Sequence, Tuple

import numpy as np

from ._native import check, lib

ARENA_BYTES = 65536  # ENET_RANGE_ARENA_BYTES
DEFAULT_WORKERS = 65536  # concurrent coders (lanes) per launch; 4 GiB of arena scratch


def gather_slices(in_buffers: Sequence) -> bytes:
    """The byte sequence compress.rs:103-126 codes for a slice list: the slices in
    order, except that an empty slice after the first reads as one 0 byte (Rust's
    dangling empty-slice pointer, compress.rs:119-122 with c.rs:79-85)."""
    parts = []
    for i, b in enumerate(in_buffers):
        b = bytes(b)
        if len(b) == 0 and i > 0:
            parts.append(b"\x00")
        else:
            parts.append(b)
    return b"".join(parts)


_scratch = {}


def _scratch_for(dev, stream, workers: int):
    """Arena scratch for `workers` coders, one buffer per (device, stream), grown on
    demand.  Launches on one stream run in order, so they can share a buffer; launches
    on different streams get different buffers (no race on the arenas).  A buffer that
    is replaced is marked as used by its stream first, so torch's caching allocator does
    not hand it out again while a launch on that stream may still be reading it."""
    import torch

    need = int(lib().enet_range_scratch_bytes(workers))
    key = (str(dev), int(stream.cuda_stream))
    buf = _scratch.get(key)
    if buf is None or buf.numel() < need:
        old = _scratch.pop(key, None)
        if old is not None:
            old.record_stream(stream)
        with torch.cuda.stream(stream):
            buf = torch.empty(need, dtype=torch.uint8, device=dev)
        _scratch[key] = buf
    return buf[:need]


def _run(decompress: bool, data, in_offsets, in_lengths, out_offsets, out_limits, out_bytes: int,
         workers: Optional[int], stream):
    import torch

    dev = data.device
    if not data.is_cuda or data.dtype != torch.uint8 or not data.is_contiguous():
        raise ValueError("data must be a contiguous uint8 device tensor")
    if stream is None:
        stream = torch.cuda.current_stream(dev)
    elif stream.device != dev:
        raise ValueError("stream must belong to the data's device")
    n = int(in_lengths.numel())
    with torch.cuda.stream(stream):
        out = torch.empty(max(out_bytes, 1), dtype=torch.uint8, device=dev)
        sizes = torch.empty(n, dtype=torch.int32, device=dev)
    if n == 0:
        return out, sizes
    w = min(n, workers or DEFAULT_WORKERS)
    scratch = _scratch_for(dev, stream, w)
    for t, dt in ((in_offsets, torch.int64), (in_lengths, torch.int32), (out_offsets, torch.int64),
                  (out_limits, torch.int32)):
        if t.device != dev or t.dtype != dt or not t.is_contiguous() or t.numel() != n:
            raise ValueError("offsets must be contiguous int64 and lengths/limits int32 on the data's device, "
                             "one entry per packet")
    fn = lib().enet_range_decompress_ragged_device if decompress else lib().enet_range_compress_ragged_device
    check(fn(data.data_ptr(), in_offsets.data_ptr(), in_lengths.data_ptr(), n, out.data_ptr(),
             out_offsets.data_ptr(), out_limits.data_ptr(), sizes.data_ptr(), scratch.data_ptr(),
             scratch.numel(), stream.cuda_stream),
          "enet_range_decompress_ragged_device" if decompress else "enet_range_compress_ragged_device")
    return out, sizes


def _default_out_layout(limits):
    import torch

    offsets = torch.zeros_like(limits, dtype=torch.int64)
    if limits.numel() > 1:
        offsets[1:] = torch.cumsum(limits[:-1].to(torch.int64), 0)
    total = int(limits.to(torch.int64).sum().item()) if limits.numel() else 0
    return offsets, total


def compress_batch(data, in_offsets, in_lengths, out_limits=None, workers: Optional[int] = None,
                   stream=None) -> Tuple["object", "object", "object"]:
    """Compress packet p = data[in_offsets[p] : +in_lengths[p]] (device tensors) into
    its own output window (limit out_limits[p], default = in_lengths[p], i.e. the send
    path's limit, protocol.rs:2228-2235).  Returns (out, out_offsets, sizes): packet p's
    coded bytes are out[out_offsets[p] : +sizes[p]]; sizes[p] == 0 = not coded."""
    import torch

    if out_limits is None:
        out_limits = in_lengths.to(device=data.device, dtype=torch.int32)
    out_offsets, total = _default_out_layout(out_limits)
    out, sizes = _run(False, data, in_offsets, in_lengths, out_offsets, out_limits, total, workers, stream)
    return out, out_offsets, sizes


def decompress_batch(data, in_offsets, in_lengths, out_limits, workers: Optional[int] = None,
                     stream=None) -> Tuple["object", "object", "object"]:
    """Decompress packet p (device tensors) into a window of out_limits[p] bytes
    (the receive path uses 4096 - header_size, protocol.rs:1450-1455)."""
    out_offsets, total = _default_out_layout(out_limits)
    out, sizes = _run(True, data, in_offsets, in_lengths, out_offsets, out_limits, total, workers, stream)
    return out, out_offsets, sizes


class RangeCoder:
    """``RangeCoder`` (src/compressor.rs:17-69) on the GPU.  ``compress`` and
    ``decompress`` follow the `Compressor` trait: they write into ``out`` (a writable
    buffer: bytearray, numpy array, memoryview) and return the byte count.  Backed by
    a context's host-memory entry points (the context owns the arena scratch)."""

    def __init__(self, device: int = 0, ctx=None):
        from .checksum import Context

        self.ctx = ctx if ctx is not None else Context(device)

    def compress(self, in_buffers: Sequence, in_limit: int, out) -> int:
        """compressor.rs:38-57 / compress.rs:60-462."""
        return self.ctx.range_compress(in_buffers, in_limit, out)

    def decompress(self, in_data, out) -> int:
        """compressor.rs:59-68 / compress.rs:463-987."""
        return self.ctx.range_decompress(in_data, out)
