// Batched checksum-slot fix-up for ENet receive-verify and send-insert (gfx950).
//
// After the ragged CRC kernels have checksummed a batch of datagrams AS STORED (the
// slot holding whatever it holds), one thread per datagram applies the linear slot
// correction of crc32_slot.hpp:
//   verify (src/c/protocol.rs:1470-1502): desired = the slot's u32 as received;
//     crc = checksum with slot := slot_value (connect_id or 0); ok = crc == desired.
//   insert (src/c/protocol.rs:2255-2293): crc = checksum with slot := slot_value;
//     the slot is then overwritten with crc (native-endian, like :2288-2292).
// The operator ladder levels a block needs are staged in LDS (one block-wide max over
// its datagrams' trailing-byte counts decides how many); the rest stay in global memory.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "crc32_kernels.hpp"
#include "crc32_slot.hpp"

namespace enet_crc {

namespace {

constexpr int kFixBlock = 256;
constexpr int kFixLdsLevels = 12;  // 48 KiB: datagrams with < 16 KiB after the slot

struct SlotBatch {
  uint8_t* base;
  const uint64_t* offsets;
  const uint32_t* lengths;
  const uint32_t* slot_offsets;
  const uint32_t* slot_values;
  uint64_t count;
  uint32_t* crc;  // in: checksum of the datagram as stored; out: with slot := slot_value
  uint32_t* ok;   // verify: 1 = accept, 0 = drop
  const uint32_t* ladder;  // kSlotLevels levels, global memory
};

__device__ __forceinline__ uint32_t load_u32_bytes(const uint8_t* p) {
  return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}

template <bool kInsert>
__global__ __launch_bounds__(kFixBlock) void crc32_slot_fixup_kernel(SlotBatch b) {
  __shared__ uint32_t lad[kFixLdsLevels * kSlotLevelDwords];
  __shared__ int need;
  if (threadIdx.x == 0) need = 1;
  __syncthreads();
  const uint64_t stride = (uint64_t)gridDim.x * kFixBlock;
  int mine = 1;
  for (uint64_t p = (uint64_t)blockIdx.x * kFixBlock + threadIdx.x; p < b.count; p += stride) {
    const uint32_t len = b.lengths[p], so = b.slot_offsets[p];
    if (so <= len && len - so >= 4) mine = max(mine, slot_levels_for(len - so - 4));
  }
  if (mine > 1) atomicMax(&need, mine);
  __syncthreads();
  const int levels = min(need, kFixLdsLevels);
  for (uint32_t x = threadIdx.x; x < (uint32_t)levels * kSlotLevelDwords; x += kFixBlock) lad[x] = b.ladder[x];
  __syncthreads();
  for (uint64_t p = (uint64_t)blockIdx.x * kFixBlock + threadIdx.x; p < b.count; p += stride) {
    const uint32_t len = b.lengths[p], so = b.slot_offsets[p];
    const uint32_t raw = b.crc[p];
    if (so > len || len - so < 4) {  // no slot inside the datagram: nothing to verify or write
      if constexpr (!kInsert) b.ok[p] = 0u;
      continue;
    }
    uint8_t* slot = b.base + b.offsets[p] + so;
    const uint32_t stored = load_u32_bytes(slot), v = b.slot_values[p];
    const uint32_t crc = raw ^ slot_delta(lad, levels, b.ladder, stored ^ v, len - so - 4);
    b.crc[p] = crc;
    if constexpr (kInsert) {
      slot[0] = (uint8_t)crc;
      slot[1] = (uint8_t)(crc >> 8);
      slot[2] = (uint8_t)(crc >> 16);
      slot[3] = (uint8_t)(crc >> 24);
    } else {
      b.ok[p] = crc == stored ? 1u : 0u;
    }
  }
}

}  // namespace

hipError_t launch_slot_fixup(bool insert, uint8_t* base, const uint64_t* offsets, const uint32_t* lengths,
                             const uint32_t* slot_offsets, const uint32_t* slot_values, uint64_t count,
                             uint32_t* crc, uint32_t* ok, const uint32_t* ladder, hipStream_t stream) {
  if (count == 0) return hipSuccess;
  const int cus = cu_count_for_current_device();
  if (cus <= 0) return hipErrorNoDevice;
  uint64_t blocks = (count + kFixBlock - 1) / kFixBlock;
  if (blocks > (uint64_t)cus * 4) blocks = (uint64_t)cus * 4;
  const SlotBatch sb{base, offsets, lengths, slot_offsets, slot_values, count, crc, ok, ladder};
  if (insert)
    hipLaunchKernelGGL(crc32_slot_fixup_kernel<true>, dim3((unsigned)blocks), dim3(kFixBlock), 0, stream, sb);
  else
    hipLaunchKernelGGL(crc32_slot_fixup_kernel<false>, dim3((unsigned)blocks), dim3(kFixBlock), 0, stream, sb);
  return hipGetLastError();
}

}  // namespace enet_crc
