"""Host-side mirror of rusty_enet's `Compressor` / `RangeCoder`, backed by the gfx950 kernels.

Reference interface (jabuwu/rusty_enet v0.4.0, src/compressor.rs):
  * ``trait Compressor { fn compress(&mut self, in_buffers: &[&[u8]], in_limit: usize,
    out: &mut [u8]) -> usize; fn decompress(&mut self, in_data: &[u8], out: &mut [u8]) -> usize; }``
    (:9-14)
  * ``RangeCoder::new()`` (:22-28) and its impl (:36-69) over src/c/compress.rs.

``RangeCoder.compress`` / ``.decompress`` take the same arguments and return the same
sizes (0 = not compressible within ``len(out)`` / malformed stream).  They run one
packet through the batched device entry points, so they pay a launch and two PCIe
copies per call; ``compress_batch`` / ``decompress_batch`` are the real interface
(one launch for a whole batch of datagrams, include/enet_range_amd.h).  There is no
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


def _scratch_for(dev, workers: int):
    """Arena scratch for `workers` coders: one pool per device, grown on demand and
    shared by the launches of this process (they run in stream order on the caller's
    stream; concurrent launches on different streams need their own scratch)."""
    import torch

    need = int(lib().enet_range_scratch_bytes(workers))
    buf = _scratch.get(str(dev))
    if buf is None or buf.numel() < need:
        _scratch.pop(str(dev), None)
        buf = torch.empty(need, dtype=torch.uint8, device=dev)
        _scratch[str(dev)] = buf
    return buf[:need]


def _run(decompress: bool, data, in_offsets, in_lengths, out_offsets, out_limits, out_bytes: int,
         workers: Optional[int], stream):
    import torch

    dev = data.device
    n = int(in_lengths.numel())
    out = torch.empty(max(out_bytes, 1), dtype=torch.uint8, device=dev)
    sizes = torch.empty(n, dtype=torch.int32, device=dev)
    if n == 0:
        return out, sizes
    w = min(n, workers or DEFAULT_WORKERS)
    scratch = _scratch_for(dev, w)
    for t, dt in ((in_offsets, torch.int64), (in_lengths, torch.int32), (out_offsets, torch.int64),
                  (out_limits, torch.int32)):
        if t.device != dev or t.dtype != dt or not t.is_contiguous():
            raise ValueError("offsets must be contiguous int64 and lengths/limits int32 on the data's device")
    if stream is None:
        stream = torch.cuda.current_stream(dev).cuda_stream
    fn = lib().enet_range_decompress_ragged_device if decompress else lib().enet_range_compress_ragged_device
    check(fn(data.data_ptr(), in_offsets.data_ptr(), in_lengths.data_ptr(), n, out.data_ptr(),
             out_offsets.data_ptr(), out_limits.data_ptr(), sizes.data_ptr(), scratch.data_ptr(),
             scratch.numel(), stream),
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
    buffer: bytearray, numpy array, memoryview) and return the byte count."""

    def __init__(self, device: int = 0):
        import torch

        self.dev = torch.device("cuda", device)

    def _one(self, decompress: bool, payload: bytes, out) -> int:
        import torch

        view = memoryview(out).cast("B")
        limit = len(view)
        src = torch.from_numpy(np.frombuffer(payload or b"\x00", dtype=np.uint8).copy()).to(self.dev)
        offs = torch.zeros(1, dtype=torch.int64, device=self.dev)
        lens = torch.tensor([len(payload)], dtype=torch.int32, device=self.dev)
        lims = torch.tensor([limit], dtype=torch.int32, device=self.dev)
        res, sizes = _run(decompress, src, offs, lens, offs, lims, limit, 1, None)
        n = int(sizes.cpu()[0])
        if n:
            view[:n] = res[:n].cpu().numpy().tobytes()
        return n

    def compress(self, in_buffers: Sequence, in_limit: int, out) -> int:
        """compressor.rs:38-57 / compress.rs:60-462.  ``in_limit`` only gates an empty
        call (compress.rs:79), as in the reference."""
        if len(in_buffers) == 0 or in_limit <= 0:
            return 0
        return self._one(False, gather_slices(in_buffers), out)

    def decompress(self, in_data, out) -> int:
        """compressor.rs:59-68 / compress.rs:463-987."""
        payload = bytes(in_data)
        if len(payload) == 0:
            return 0
        return self._one(True, payload, out)
