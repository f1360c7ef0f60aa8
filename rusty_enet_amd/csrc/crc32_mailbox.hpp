// Persistent per-call checksum server (ENET_CRC_PERCALL_PERSISTENT, enet_crc32_iov):
// one wave polls a request mailbox (in device memory the host writes through the BAR, or
// in pinned host memory), checksums each datagram the host posts there and writes the
// register back into pinned host memory, so a call costs PCIe transfers instead of a
// kernel launch plus a stream synchronisation.  Shared by
// crc32_mailbox.hip (the kernel) and enet_crc_abi.hip (the host side).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace enet_crc {

constexpr uint32_t kMailboxBytes = 4096;         // largest datagram served (PROTOCOL_MAXIMUM_MTU)
constexpr uint32_t kMailboxStop = 0xFFFFFFFFu;   // seq value that makes the server exit
constexpr uint64_t kMailboxIdleTicks = 2000000;  // 20 ms of the 100-MHz wall clock without a request: exit
constexpr uint64_t kMailboxMaxTicks = 200000000; // 2 s: exit (the host relaunches on the next call)

// Host and device view of the mailbox; the three groups of fields sit on separate lines.
// seq/len and done/result are each written with one 64-bit store and read with one
// 64-bit load (one PCIe round trip each).
struct alignas(128) Mailbox {
  uint32_t seq;  // host -> server: number of the posted request (kMailboxStop: exit)
  uint32_t len;  // bytes of the posted request, right-aligned at the end of data
  uint32_t pad0[30];
  uint32_t done;    // server -> host: number of the last request served
  uint32_t result;  // its zero-initialised register (the initial register is added on the host)
  uint32_t pad1[30];
  uint8_t data[kMailboxBytes];  // request bytes end at data + kMailboxBytes; the 64-B chunk
                                // holding the first byte is zero below it
};

// Starts the server wave on `stream`.  `req` is the device address of the mailbox the
// requests are read from (seq, len, data: fine-grained device memory the host writes
// through the PCIe BAR when the device has a large BAR, else pinned host memory), `resp`
// that of the one the answers go to (done, result: always pinned host memory, where the
// host polls); `ladder` is the device ladder of crc32_slot.hpp.  The kernel returns on
// kMailboxStop, after kMailboxIdleTicks without a request, after kMailboxMaxTicks, or when
// the device's kick word changes.
// `kick` is the device's kick word (enet_crc_abi.hip): the first workgroup of every batch
// kernel on the device bumps it, and the server exits as soon as it reads another value than
// at its start, so the CU it holds is free for the batch's grid.
hipError_t launch_mailbox(const Mailbox* req, Mailbox* resp, const uint32_t* ladder, const uint32_t* kick,
                          hipStream_t stream);

}  // namespace enet_crc
