"""rusty_enet_amd: MI355X-native (gfx950 HIP) ENet per-datagram CRC-32.

Drop-in for the checksum path of jabuwu/rusty_enet (src/crc32.rs and the
HostSettings::checksum hook, src/host.rs:40), plus the batched range coder
(the `Compressor` RangeCoder, src/compressor.rs, src/c/compress.rs).  See DESIGN.md / INTEGRATION.md.
"""
from ._native import CrcError, NativeLibraryMissing, LIB_PATH, HEADER_PATH  # noqa: F401
from .checksum import (  # noqa: F401
    Context,
    checksum_fn,
    crc32,
    crc32_batch,
    crc32_combine,
    crc32_ragged_device,
    crc32_shards_device,
    crc32_uniform_device,
    default_context,
    device_status,
    insert_batch,
    shard_bounds_native,
    slot_adjust,
    verify_batch,
)

from .range_coder import RangeCoder, compress_batch, decompress_batch, gather_slices  # noqa: F401

__all__ = [
    "Context", "CrcError", "NativeLibraryMissing", "checksum_fn", "crc32", "crc32_batch", "crc32_combine",
    "crc32_ragged_device", "crc32_shards_device", "crc32_uniform_device", "shard_bounds_native", "default_context", "device_status", "insert_batch", "slot_adjust",
    "verify_batch", "RangeCoder", "compress_batch", "decompress_batch", "gather_slices",
]
