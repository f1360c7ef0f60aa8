// Internal launcher interface between the C ABI (enet_crc_abi.hip) and the
// gfx950 kernels (crc32_kernels.hip).  Not part of the public ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace enet_crc {

// Packets p = 0..count-1 at base + p*stride, each `length` bytes.
hipError_t launch_uniform(const uint8_t* base, uint64_t stride, uint32_t length, uint64_t count,
                          uint32_t* out, hipStream_t stream);

// One packet of `length` bytes at `base`, any memory the device can read (the per-call
// path passes mapped pinned host memory), result to `out` (may be mapped host memory).
// Register-staged loads only (no LDS-DMA from host memory).
hipError_t launch_single(const uint8_t* base, uint32_t length, uint32_t* out, hipStream_t stream);

// Packets p at base + offsets[p], lengths[p] bytes (device arrays).
hipError_t launch_ragged(const uint8_t* base, const uint64_t* offsets, const uint32_t* lengths,
                         uint64_t count, uint32_t* out, hipStream_t stream);

// Slot fix-up after a ragged checksum pass (crc32_slot.hip): crc[p] holds the checksum
// of datagram p as stored; afterwards the checksum with its 4-byte slot at
// slot_offsets[p] set to slot_values[p].  insert: that checksum is written into the
// slot; verify: ok[p] = (it equals the slot's stored u32).  `ladder`: device copy of
// build_slot_ladder().
hipError_t launch_slot_fixup(bool insert, uint8_t* base, const uint64_t* offsets, const uint32_t* lengths,
                             const uint32_t* slot_offsets, const uint32_t* slot_values, uint64_t count,
                             uint32_t* crc, uint32_t* ok, const uint32_t* ladder, hipStream_t stream);

// Device copy of the operator ladder (crc32_slot.hpp: build_slot_ladder, then
// build_inverse_ladder) for the calling thread's device, uploaded on first use.
hipError_t device_slot_ladder(const uint32_t** out);

// Cached hipDeviceAttributeMultiprocessorCount of the calling thread's device.
int cu_count_for_current_device();

// Registers the current device's kick word (enet_crc_abi.hip) with its batch kernels.
hipError_t set_device_kick_word(uint32_t* d_word);

// Host address of device `dev`'s failure word (mapped, coherent pinned memory; allocated
// and registered with that device's kernels on first use).  Non-zero once a batch kernel
// gave up on an inter-wave wait (crc32_ragged_jobs_kernel: kFault* bits); sticky until
// the host writes 0.  launch_ragged calls it before every launch.
hipError_t device_fault_word(int dev, volatile uint32_t** host_word);

}  // namespace enet_crc
