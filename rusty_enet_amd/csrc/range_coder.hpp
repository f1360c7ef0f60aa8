// Internal launcher interface of the range-coder kernels (range_coder.hip).
// Not part of the public ABI (that is include/enet_range_amd.h).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace enet_crc {

// One coder's symbol arena: 4096 ENetSymbol of 16 B (reference src/c/compress.rs:7-9).
constexpr uint64_t kRangeArenaBytes = 4096 * 16;

// Batched per-packet compress (decompress = false) or decompress (true).  Packet p is
// in_len[p] bytes at in + in_off[p]; its output goes to out + out_off[p], at most
// out_lim[p] bytes; the coder's return value goes to sizes[p].  `scratch` holds
// `workers` arenas (kRangeArenaBytes each, 16-B aligned); one lane = one coder.
hipError_t launch_range(bool decompress, const uint8_t* in, const uint64_t* in_off, const uint32_t* in_len,
                        uint64_t count, uint8_t* out, const uint64_t* out_off, const uint32_t* out_lim,
                        uint32_t* sizes, void* scratch, uint64_t workers, hipStream_t stream);

}  // namespace enet_crc
