/*
 * enet_range_amd.h -- C ABI of the batched ENet range coder on MI355X (gfx950).
 * Part of libenet_crc_amd.so; status codes and ENET_CRC_API from enet_crc_amd.h.
 *
 * Replaces, for a batch of packets, the per-datagram calls of the `Compressor`
 * trait implemented by `RangeCoder` in jabuwu/rusty_enet v0.4.0:
 *   - src/compressor.rs:38  fn compress(&mut self, in_buffers: &[&[u8]], in_limit: usize, out: &mut [u8]) -> usize
 *       -> enet_range_coder_compress, src/c/compress.rs:60-462;
 *          called by the send path, src/c/protocol.rs:2213-2242
 *   - src/compressor.rs:59  fn decompress(&mut self, in_data: &[u8], out: &mut [u8]) -> usize
 *       -> enet_range_coder_decompress, src/c/compress.rs:463-987;
 *          called by the receive path, src/c/protocol.rs:1442-1468
 *
 * Each packet is coded independently with a fresh model, exactly as one call of
 * the reference does (every call re-initialises the arena, compress.rs:86-101 /
 * :484-499).  Output bytes and sizes equal the reference's for the same input:
 * size 0 means what it means there (empty input, output limit reached, or a
 * malformed stream on decompress).
 *
 * A packet given here is ONE contiguous slice.  The send path's slice list
 * (header + payload segments) is gathered first; the reference reads an EMPTY
 * slice in the middle of that list as a single 0 byte (compress.rs:119-122 with
 * c.rs:79-85), so a caller gathering such a list inserts that byte
 * (rusty_enet_amd.range_coder.gather_slices does).
 */
#ifndef ENET_RANGE_AMD_H
#define ENET_RANGE_AMD_H

#include "enet_crc_amd.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Bytes of device scratch per concurrent coder: one 4096 x 16-B symbol arena
 * (ENetRangeCoder, src/c/compress.rs:7-9). */
#define ENET_RANGE_ARENA_BYTES 65536u

/* Scratch bytes that let `workers` coders run at once (workers x the arena). */
ENET_CRC_API uint64_t enet_range_scratch_bytes(uint64_t workers);

/*
 * Batched compress, device-resident.  Packet p is d_in_lengths[p] bytes at
 * d_in + d_in_offsets[p]; its compressed bytes go to d_out + d_out_offsets[p],
 * at most d_out_limits[p] of them (the reference's `out.len()`; the send path
 * passes the uncompressed size, protocol.rs:2228-2235).  d_sizes[p] = the
 * return value of compress() for that packet.  `d_scratch` holds
 * scratch_bytes / ENET_RANGE_ARENA_BYTES coder arenas (16-B aligned, >= 1);
 * that many packets are coded concurrently.  Asynchronous on `hip_stream`.
 */
ENET_CRC_API int enet_range_compress_ragged_device(const void* d_in, const uint64_t* d_in_offsets,
                                                   const uint32_t* d_in_lengths, uint64_t count, void* d_out,
                                                   const uint64_t* d_out_offsets, const uint32_t* d_out_limits,
                                                   uint32_t* d_sizes, void* d_scratch, uint64_t scratch_bytes,
                                                   void* hip_stream);

/*
 * Batched decompress, same layout: packet p's compressed bytes in, its
 * decompressed bytes out (limit d_out_limits[p]; the receive path passes
 * 4096 - header_size, protocol.rs:1450-1455), d_sizes[p] = the return value of
 * decompress() (0 = drop the datagram, :1456-1460).
 */
ENET_CRC_API int enet_range_decompress_ragged_device(const void* d_in, const uint64_t* d_in_offsets,
                                                     const uint32_t* d_in_lengths, uint64_t count, void* d_out,
                                                     const uint64_t* d_out_offsets, const uint32_t* d_out_limits,
                                                     uint32_t* d_sizes, void* d_scratch, uint64_t scratch_bytes,
                                                     void* hip_stream);

/*
 * Host-memory drop-ins for the `Compressor` methods (src/compressor.rs:9-14, :36-69),
 * on lane 0 of an enet_crc_ctx (the context owns the arenas and the staging).
 *
 * enet_range_compress_iov: `compress(&mut self, in_buffers, in_limit, out)`.  The
 * slices are coded as the byte sequence compress.rs:103-126 reads (an empty slice
 * after the first is one 0 byte, see above); in_limit == 0 or nbufs == 0 codes
 * nothing (compress.rs:79).  *out_size = the reference's return value (0 = not
 * coded within out_limit).  Only the first *out_size bytes of `out` are written.
 *
 * enet_range_decompress: `decompress(&mut self, in_data, out)`; *out_size = the
 * reference's return value (0 = empty input or malformed stream, or out_limit
 * reached).  Synchronous.
 */
ENET_CRC_API int enet_range_compress_iov(enet_crc_ctx* ctx, const enet_crc_iov* bufs, size_t nbufs,
                                         size_t in_limit, uint8_t* out, size_t out_limit, size_t* out_size);
ENET_CRC_API int enet_range_decompress(enet_crc_ctx* ctx, const uint8_t* in, size_t in_len, uint8_t* out,
                                       size_t out_limit, size_t* out_size);

/*
 * Host-memory batches (a receive/send batch of datagrams in one launch): the same
 * layout as the device entry points above, in host memory.  Only the first
 * h_sizes[p] bytes of packet p's output window are written.  Synchronous.
 */
ENET_CRC_API int enet_range_compress_ragged_host(enet_crc_ctx* ctx, const void* h_in, const uint64_t* h_in_offsets,
                                                 const uint32_t* h_in_lengths, uint64_t count, void* h_out,
                                                 const uint64_t* h_out_offsets, const uint32_t* h_out_limits,
                                                 uint32_t* h_sizes);
ENET_CRC_API int enet_range_decompress_ragged_host(enet_crc_ctx* ctx, const void* h_in,
                                                   const uint64_t* h_in_offsets, const uint32_t* h_in_lengths,
                                                   uint64_t count, void* h_out, const uint64_t* h_out_offsets,
                                                   const uint32_t* h_out_limits, uint32_t* h_sizes);

#ifdef __cplusplus
}
#endif

#endif /* ENET_RANGE_AMD_H */
