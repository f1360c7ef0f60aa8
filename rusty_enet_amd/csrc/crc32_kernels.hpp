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

// Packets p at base + offsets[p], lengths[p] bytes (device arrays).  `fault`: device
// address of the failure word this launch reports a give-up into (FaultWord::dev); NULL:
// the device-wide word of the stream's device (device_fault_word).
hipError_t launch_ragged(const uint8_t* base, const uint64_t* offsets, const uint32_t* lengths,
                         uint64_t count, uint32_t* out, hipStream_t stream, uint32_t* fault = nullptr);

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

// A failure word: 64 B of mapped, coherent pinned host memory.  Non-zero once a ragged jobs
// launch that carried it gave up on an inter-wave wait (crc32_ragged_jobs_kernel: kFault*
// bits); sticky until the host writes 0.
struct FaultWord {
  volatile uint32_t* host = nullptr;
  uint32_t* dev = nullptr;  // device address (hipHostGetDevicePointer)
};
// A private word (one slot of a synchronous entry: only that slot's launches write it).
hipError_t alloc_fault_word(FaultWord* w);
void free_fault_word(FaultWord& w);
// Device `dev`'s word, carried by the launches of the asynchronous *_device entries
// (allocated on first use, never freed); read by enet_crc_device_status.
hipError_t device_fault_word(int dev, FaultWord* w);

}  // namespace enet_crc
