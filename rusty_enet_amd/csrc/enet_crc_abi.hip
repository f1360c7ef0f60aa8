// C ABI of the MI355X CRC-32 path (include/enet_crc_amd.h).
//
// The reference hook is a synchronous `Fn(&[&[u8]]) -> u32` called on the
// thread running Host::service()/flush() (src/host.rs:185-201, src/c/protocol.rs
// :1499 and :2287).  This file maps that surface and the batch entry points
// onto the gfx950 kernels in crc32_kernels.hip.  There is no CPU path: every
// checksum comes from the GPU or the call returns an error.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <mutex>
#include <new>
#include <vector>

#include "../../include/enet_crc_amd.h"
#include "crc32_kernels.hpp"
#include "crc32_slot.hpp"
#include "range_coder.hpp"
#include "../../include/enet_range_amd.h"

namespace enet_crc {

namespace {

thread_local int t_last_hip_error = 0;

int fail_hip(hipError_t e) {
  t_last_hip_error = (int)e;
  if (e == hipErrorNoDevice || e == hipErrorInvalidDevice) return ENET_CRC_E_NO_DEVICE;
  if (e == hipErrorOutOfMemory) return ENET_CRC_E_NOMEM;
  return ENET_CRC_E_HIP;
}

#define ENET_HIP_TRY(expr)                 \
  do {                                     \
    hipError_t _e = (expr);                \
    if (_e != hipSuccess) return fail_hip(_e); \
  } while (0)

constexpr int kMaxDevices = 64;
std::atomic<int> g_cu_count[kMaxDevices];

// Restores the caller's current device on scope exit.
struct DeviceGuard {
  int prev = -1;
  explicit DeviceGuard(int dev) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    if (prev != dev) (void)hipSetDevice(dev);
  }
  ~DeviceGuard() {
    int cur = -1;
    if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
  }
};

}  // namespace

// Operator ladder of the slot correction (crc32_slot.hpp): one host copy, one device
// copy per device (uploaded on first use, never freed: 128 KiB).
const uint32_t* host_slot_ladder() {
  static uint32_t* ladder = [] {
    uint32_t* l = new uint32_t[kSlotLevels * kSlotLevelDwords];
    build_slot_ladder(l);
    return l;
  }();
  return ladder;
}

std::mutex g_ladder_lock;
uint32_t* g_device_ladder[kMaxDevices];

hipError_t device_slot_ladder(const uint32_t** out) {
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return e;
  if (dev < 0 || dev >= kMaxDevices) return hipErrorInvalidDevice;
  std::lock_guard<std::mutex> lk(g_ladder_lock);
  if (!g_device_ladder[dev]) {
    const size_t bytes = sizeof(uint32_t) * kSlotLevels * kSlotLevelDwords;
    uint32_t* d = nullptr;
    e = hipMalloc((void**)&d, bytes);
    if (e != hipSuccess) return e;
    e = hipMemcpy(d, host_slot_ladder(), bytes, hipMemcpyHostToDevice);
    if (e != hipSuccess) {
      (void)hipFree(d);
      return e;
    }
    g_device_ladder[dev] = d;
  }
  *out = g_device_ladder[dev];
  return hipSuccess;
}

int cu_count_for_current_device() {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kMaxDevices) return -1;
  int n = g_cu_count[dev].load(std::memory_order_relaxed);
  if (n > 0) return n;
  if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return -1;
  g_cu_count[dev].store(n, std::memory_order_relaxed);
  return n;
}

}  // namespace enet_crc

using namespace enet_crc;

// One pipeline slot of the host path: pinned input bytes + descriptors, device
// copies, pinned output.
struct StageSlot {
  uint8_t* h_bytes = nullptr;
  uint64_t* h_offsets = nullptr;
  uint32_t* h_lengths = nullptr;
  uint32_t* h_out = nullptr;
  uint8_t* d_bytes = nullptr;
  uint64_t* d_offsets = nullptr;
  uint32_t* d_lengths = nullptr;
  uint32_t* d_out = nullptr;
  size_t byte_cap = 0;
  size_t pkt_cap = 0;
  hipStream_t stream = nullptr;
  hipEvent_t done = nullptr;
  uint64_t first = 0;  // packet range staged in this slot
  uint64_t n = 0;
  bool busy = false;
};

struct enet_crc_ctx {
  int device = 0;
  std::mutex lock;
  StageSlot slot[2];
};

// One slot of a pinned receive ring (include/enet_crc_amd.h).
struct RingSlot {
  uint8_t* h_data = nullptr;
  uint64_t* h_offsets = nullptr;
  uint32_t* h_lengths = nullptr;
  uint32_t* h_crcs = nullptr;
  uint8_t* d_data = nullptr;
  uint64_t* d_offsets = nullptr;
  uint32_t* d_lengths = nullptr;
  uint32_t* d_crcs = nullptr;
  hipStream_t stream = nullptr;
  hipEvent_t done = nullptr;
  bool busy = false;
};

struct enet_crc_ring {
  int device = 0;
  uint64_t slot_bytes = 0;
  uint32_t slot_packets = 0;
  std::mutex lock;  // guards the busy flags; never held across a device wait
  std::vector<RingSlot> slots;
};

namespace {

void free_slot_buffers(StageSlot& s) {
  if (s.h_bytes) (void)hipHostFree(s.h_bytes);
  if (s.h_offsets) (void)hipHostFree(s.h_offsets);
  if (s.h_lengths) (void)hipHostFree(s.h_lengths);
  if (s.h_out) (void)hipHostFree(s.h_out);
  if (s.d_bytes) (void)hipFree(s.d_bytes);
  if (s.d_offsets) (void)hipFree(s.d_offsets);
  if (s.d_lengths) (void)hipFree(s.d_lengths);
  if (s.d_out) (void)hipFree(s.d_out);
  s.h_bytes = nullptr; s.h_offsets = nullptr; s.h_lengths = nullptr; s.h_out = nullptr;
  s.d_bytes = nullptr; s.d_offsets = nullptr; s.d_lengths = nullptr; s.d_out = nullptr;
  s.byte_cap = 0; s.pkt_cap = 0;
}

// Grows the slot to hold `bytes` input bytes and `pkts` packets (caller holds the ctx lock,
// the slot is idle).
int reserve_slot(StageSlot& s, size_t bytes, size_t pkts) {
  bytes = std::max<size_t>(bytes, 4096);
  pkts = std::max<size_t>(pkts, 64);
  if (bytes > s.byte_cap) {
    if (s.h_bytes) (void)hipHostFree(s.h_bytes);
    if (s.d_bytes) (void)hipFree(s.d_bytes);
    s.h_bytes = nullptr; s.d_bytes = nullptr; s.byte_cap = 0;
    // +16: the kernel's 4-byte-grid loads never cross the packet's own words,
    // but keep the staging allocation a whole number of 16-byte lines.
    const size_t alloc = (bytes + 16 + 15) & ~(size_t)15;
    ENET_HIP_TRY(hipHostMalloc((void**)&s.h_bytes, alloc, hipHostMallocDefault));
    ENET_HIP_TRY(hipMalloc((void**)&s.d_bytes, alloc));
    s.byte_cap = bytes;
  }
  if (pkts > s.pkt_cap) {
    if (s.h_offsets) (void)hipHostFree(s.h_offsets);
    if (s.h_lengths) (void)hipHostFree(s.h_lengths);
    if (s.h_out) (void)hipHostFree(s.h_out);
    if (s.d_offsets) (void)hipFree(s.d_offsets);
    if (s.d_lengths) (void)hipFree(s.d_lengths);
    if (s.d_out) (void)hipFree(s.d_out);
    s.h_offsets = nullptr; s.h_lengths = nullptr; s.h_out = nullptr;
    s.d_offsets = nullptr; s.d_lengths = nullptr; s.d_out = nullptr; s.pkt_cap = 0;
    ENET_HIP_TRY(hipHostMalloc((void**)&s.h_offsets, pkts * sizeof(uint64_t), hipHostMallocDefault));
    ENET_HIP_TRY(hipHostMalloc((void**)&s.h_lengths, pkts * sizeof(uint32_t), hipHostMallocDefault));
    ENET_HIP_TRY(hipHostMalloc((void**)&s.h_out, pkts * sizeof(uint32_t), hipHostMallocDefault));
    ENET_HIP_TRY(hipMalloc((void**)&s.d_offsets, pkts * sizeof(uint64_t)));
    ENET_HIP_TRY(hipMalloc((void**)&s.d_lengths, pkts * sizeof(uint32_t)));
    ENET_HIP_TRY(hipMalloc((void**)&s.d_out, pkts * sizeof(uint32_t)));
    s.pkt_cap = pkts;
  }
  return ENET_CRC_OK;
}

// Host path chunking: at most this many staged bytes / packets per slot.
constexpr size_t kStageBytes = 64u << 20;
constexpr size_t kStagePackets = 1u << 18;

}  // namespace

extern "C" {

int enet_crc_abi_version(void) { return ENET_CRC_ABI_VERSION; }

const char* enet_crc_strerror(int status) {
  switch (status) {
    case ENET_CRC_OK: return "ok";
    case ENET_CRC_E_INVALID: return "invalid argument";
    case ENET_CRC_E_NO_DEVICE: return "no usable HIP device";
    case ENET_CRC_E_HIP: return "HIP runtime error";
    case ENET_CRC_E_NOMEM: return "out of memory";
    default: return "unknown status";
  }
}

int enet_crc_last_hip_error(void) { return t_last_hip_error; }

int enet_crc_device_count(void) {
  int n = 0;
  hipError_t e = hipGetDeviceCount(&n);
  if (e == hipErrorNoDevice) return 0;
  if (e != hipSuccess) return fail_hip(e);
  return n;
}

int enet_crc_ctx_create(int device, enet_crc_ctx** out_ctx) {
  if (!out_ctx) return ENET_CRC_E_INVALID;
  *out_ctx = nullptr;
  int n = 0;
  hipError_t e = hipGetDeviceCount(&n);
  if (e != hipSuccess || n <= 0) return e == hipSuccess ? ENET_CRC_E_NO_DEVICE : fail_hip(e);
  if (device < 0 || device >= n) return ENET_CRC_E_NO_DEVICE;
  enet_crc_ctx* ctx = new (std::nothrow) enet_crc_ctx();
  if (!ctx) return ENET_CRC_E_NOMEM;
  ctx->device = device;
  DeviceGuard g(device);
  for (auto& s : ctx->slot) {
    hipError_t se = hipStreamCreateWithFlags(&s.stream, hipStreamNonBlocking);
    if (se == hipSuccess) se = hipEventCreateWithFlags(&s.done, hipEventDisableTiming);
    if (se != hipSuccess) {
      enet_crc_ctx_destroy(ctx);
      return fail_hip(se);
    }
  }
  *out_ctx = ctx;
  return ENET_CRC_OK;
}

void enet_crc_ctx_destroy(enet_crc_ctx* ctx) {
  if (!ctx) return;
  {
    DeviceGuard g(ctx->device);
    for (auto& s : ctx->slot) {
      if (s.stream) (void)hipStreamSynchronize(s.stream);
      free_slot_buffers(s);
      if (s.done) (void)hipEventDestroy(s.done);
      if (s.stream) (void)hipStreamDestroy(s.stream);
    }
  }
  delete ctx;
}

int enet_crc32_uniform_device(const void* d_base, uint64_t stride, uint32_t length, uint64_t count,
                              uint32_t* d_out, void* hip_stream) {
  if (count == 0) return ENET_CRC_OK;
  if (!d_out || (!d_base && length > 0)) return ENET_CRC_E_INVALID;
  hipError_t e = launch_uniform(static_cast<const uint8_t*>(d_base), stride, length, count, d_out,
                                static_cast<hipStream_t>(hip_stream));
  return e == hipSuccess ? ENET_CRC_OK : fail_hip(e);
}

int enet_crc32_ragged_device(const void* d_base, const uint64_t* d_offsets, const uint32_t* d_lengths,
                             uint64_t count, uint32_t* d_out, void* hip_stream) {
  if (count == 0) return ENET_CRC_OK;
  if (!d_base || !d_offsets || !d_lengths || !d_out) return ENET_CRC_E_INVALID;
  hipError_t e = launch_ragged(static_cast<const uint8_t*>(d_base), d_offsets, d_lengths, count, d_out,
                               static_cast<hipStream_t>(hip_stream));
  return e == hipSuccess ? ENET_CRC_OK : fail_hip(e);
}

// Shared body of the batched verify / insert entry points: checksum the datagrams as
// stored (ragged kernels), then the slot fix-up kernel.
static int slot_batch(bool insert, uint8_t* d_base, const uint64_t* d_offsets, const uint32_t* d_lengths,
                      const uint32_t* d_slot_offsets, const uint32_t* d_slot_values, uint64_t count, uint32_t* d_crc,
                      uint32_t* d_ok, void* hip_stream) {
  if (count == 0) return ENET_CRC_OK;
  if (!d_base || !d_offsets || !d_lengths || !d_slot_offsets || !d_slot_values || !d_crc || (!insert && !d_ok))
    return ENET_CRC_E_INVALID;
  const hipStream_t stream = static_cast<hipStream_t>(hip_stream);
  const uint32_t* ladder = nullptr;
  ENET_HIP_TRY(device_slot_ladder(&ladder));
  ENET_HIP_TRY(launch_ragged(d_base, d_offsets, d_lengths, count, d_crc, stream));
  ENET_HIP_TRY(launch_slot_fixup(insert, d_base, d_offsets, d_lengths, d_slot_offsets, d_slot_values, count, d_crc,
                                 d_ok, ladder, stream));
  return ENET_CRC_OK;
}

int enet_crc32_verify_ragged_device(const void* d_base, const uint64_t* d_offsets, const uint32_t* d_lengths,
                                    const uint32_t* d_slot_offsets, const uint32_t* d_slot_values, uint64_t count,
                                    uint32_t* d_crc, uint32_t* d_ok, void* hip_stream) {
  // The verify kernel only reads the datagrams (the fix-up kernel is shared with insert).
  return slot_batch(false, static_cast<uint8_t*>(const_cast<void*>(d_base)), d_offsets, d_lengths, d_slot_offsets,
                    d_slot_values, count, d_crc, d_ok, hip_stream);
}

int enet_crc32_insert_ragged_device(void* d_base, const uint64_t* d_offsets, const uint32_t* d_lengths,
                                    const uint32_t* d_slot_offsets, const uint32_t* d_slot_values, uint64_t count,
                                    uint32_t* d_crc, void* hip_stream) {
  return slot_batch(true, static_cast<uint8_t*>(d_base), d_offsets, d_lengths, d_slot_offsets, d_slot_values, count,
                    d_crc, nullptr, hip_stream);
}

uint32_t enet_crc32_slot_adjust(uint32_t crc, uint32_t old_slot, uint32_t new_slot, uint32_t bytes_after_slot) {
  const uint32_t* l = host_slot_ladder();
  return crc ^ slot_delta(l, kSlotLevels, l, old_slot ^ new_slot, bytes_after_slot);
}

int enet_crc32_iov(enet_crc_ctx* ctx, const enet_crc_iov* bufs, size_t nbufs, uint32_t* out_crc) {
  if (!ctx || !out_crc || (nbufs > 0 && !bufs)) return ENET_CRC_E_INVALID;
  size_t total = 0;
  for (size_t i = 0; i < nbufs; ++i) {
    if (bufs[i].len > 0 && !bufs[i].data) return ENET_CRC_E_INVALID;
    total += bufs[i].len;
  }
  if (total > 0xFFFFFFFFull) return ENET_CRC_E_INVALID;
  std::lock_guard<std::mutex> lk(ctx->lock);
  DeviceGuard g(ctx->device);
  StageSlot& s = ctx->slot[0];
  int st = reserve_slot(s, total, 1);
  if (st != ENET_CRC_OK) return st;
  size_t pos = 0;  // concatenation, src/crc32.rs:41-42
  for (size_t i = 0; i < nbufs; ++i) {
    if (bufs[i].len) memcpy(s.h_bytes + pos, bufs[i].data, bufs[i].len);
    pos += bufs[i].len;
  }
  if (total) ENET_HIP_TRY(hipMemcpyAsync(s.d_bytes, s.h_bytes, total, hipMemcpyHostToDevice, s.stream));
  ENET_HIP_TRY(launch_uniform(s.d_bytes, 0, (uint32_t)total, 1, s.d_out, s.stream));
  ENET_HIP_TRY(hipMemcpyAsync(s.h_out, s.d_out, sizeof(uint32_t), hipMemcpyDeviceToHost, s.stream));
  ENET_HIP_TRY(hipStreamSynchronize(s.stream));
  *out_crc = s.h_out[0];
  return ENET_CRC_OK;
}

int enet_crc32_ragged_host(enet_crc_ctx* ctx, const void* h_base, const uint64_t* h_offsets,
                           const uint32_t* h_lengths, uint64_t count, uint32_t* h_out) {
  if (!ctx) return ENET_CRC_E_INVALID;
  if (count == 0) return ENET_CRC_OK;
  if (!h_base || !h_offsets || !h_lengths || !h_out) return ENET_CRC_E_INVALID;
  std::lock_guard<std::mutex> lk(ctx->lock);
  DeviceGuard g(ctx->device);
  const uint8_t* base = static_cast<const uint8_t*>(h_base);

  // Drain a slot: wait for its kernel + D2H, copy checksums out.
  auto drain = [&](StageSlot& s) -> int {
    if (!s.busy) return ENET_CRC_OK;
    ENET_HIP_TRY(hipEventSynchronize(s.done));
    memcpy(h_out + s.first, s.h_out, s.n * sizeof(uint32_t));
    s.busy = false;
    return ENET_CRC_OK;
  };

  uint64_t p = 0;
  int which = 0;
  while (p < count) {
    StageSlot& s = ctx->slot[which];
    int st = drain(s);
    if (st != ENET_CRC_OK) return st;
    // Chunk [p, q): packets whose byte span [lo, hi) fits the staging size.
    uint64_t lo = h_offsets[p], hi = h_offsets[p] + h_lengths[p];
    uint64_t q = p + 1;
    while (q < count && q - p < kStagePackets) {
      const uint64_t nlo = std::min<uint64_t>(lo, h_offsets[q]);
      const uint64_t nhi = std::max<uint64_t>(hi, h_offsets[q] + h_lengths[q]);
      if (nhi - nlo > kStageBytes) break;
      lo = nlo; hi = nhi; ++q;
    }
    // Keep the device copy at the same offset mod 4 as the host bytes, so the
    // kernel sees the same word grid (not required for correctness).
    const uint64_t lo_al = lo & ~(uint64_t)3;
    const size_t span = (size_t)(hi - lo_al);
    st = reserve_slot(s, span, (size_t)(q - p));
    if (st != ENET_CRC_OK) return st;
    memcpy(s.h_bytes, base + lo_al, span);
    for (uint64_t i = p; i < q; ++i) {
      s.h_offsets[i - p] = h_offsets[i] - lo_al;
      s.h_lengths[i - p] = h_lengths[i];
    }
    const size_t n = (size_t)(q - p);
    ENET_HIP_TRY(hipMemcpyAsync(s.d_bytes, s.h_bytes, span, hipMemcpyHostToDevice, s.stream));
    ENET_HIP_TRY(hipMemcpyAsync(s.d_offsets, s.h_offsets, n * sizeof(uint64_t), hipMemcpyHostToDevice, s.stream));
    ENET_HIP_TRY(hipMemcpyAsync(s.d_lengths, s.h_lengths, n * sizeof(uint32_t), hipMemcpyHostToDevice, s.stream));
    ENET_HIP_TRY(launch_ragged(s.d_bytes, s.d_offsets, s.d_lengths, n, s.d_out, s.stream));
    ENET_HIP_TRY(hipMemcpyAsync(s.h_out, s.d_out, n * sizeof(uint32_t), hipMemcpyDeviceToHost, s.stream));
    ENET_HIP_TRY(hipEventRecord(s.done, s.stream));
    s.first = p;
    s.n = n;
    s.busy = true;
    p = q;
    which ^= 1;
  }
  for (auto& s : ctx->slot) {
    int st = drain(s);
    if (st != ENET_CRC_OK) return st;
  }
  return ENET_CRC_OK;
}

static void ring_free_slot(RingSlot& s) {
  if (s.stream) (void)hipStreamSynchronize(s.stream);
  if (s.h_data) (void)hipHostFree(s.h_data);
  if (s.h_offsets) (void)hipHostFree(s.h_offsets);
  if (s.h_lengths) (void)hipHostFree(s.h_lengths);
  if (s.h_crcs) (void)hipHostFree(s.h_crcs);
  if (s.d_data) (void)hipFree(s.d_data);
  if (s.d_offsets) (void)hipFree(s.d_offsets);
  if (s.d_lengths) (void)hipFree(s.d_lengths);
  if (s.d_crcs) (void)hipFree(s.d_crcs);
  if (s.done) (void)hipEventDestroy(s.done);
  if (s.stream) (void)hipStreamDestroy(s.stream);
  s = RingSlot{};
}

int enet_crc_ring_create(int device, uint32_t nslots, uint64_t slot_bytes, uint32_t slot_packets,
                         enet_crc_ring** out_ring) {
  if (!out_ring) return ENET_CRC_E_INVALID;
  *out_ring = nullptr;
  if (nslots == 0 || nslots > 64 || slot_bytes == 0 || slot_packets == 0) return ENET_CRC_E_INVALID;
  int n = 0;
  hipError_t e = hipGetDeviceCount(&n);
  if (e != hipSuccess || n <= 0) return e == hipSuccess ? ENET_CRC_E_NO_DEVICE : fail_hip(e);
  if (device < 0 || device >= n) return ENET_CRC_E_NO_DEVICE;
  enet_crc_ring* r = new (std::nothrow) enet_crc_ring();
  if (!r) return ENET_CRC_E_NOMEM;
  r->device = device;
  r->slot_bytes = slot_bytes;
  r->slot_packets = slot_packets;
  r->slots.resize(nslots);
  DeviceGuard g(device);
  const size_t bytes = (size_t)((slot_bytes + 16 + 15) & ~(uint64_t)15);
  for (auto& s : r->slots) {
    hipError_t se = hipStreamCreateWithFlags(&s.stream, hipStreamNonBlocking);
    if (se == hipSuccess) se = hipEventCreateWithFlags(&s.done, hipEventDisableTiming);
    if (se == hipSuccess) se = hipHostMalloc((void**)&s.h_data, bytes, hipHostMallocDefault);
    if (se == hipSuccess) se = hipHostMalloc((void**)&s.h_offsets, slot_packets * sizeof(uint64_t), hipHostMallocDefault);
    if (se == hipSuccess) se = hipHostMalloc((void**)&s.h_lengths, slot_packets * sizeof(uint32_t), hipHostMallocDefault);
    if (se == hipSuccess) se = hipHostMalloc((void**)&s.h_crcs, slot_packets * sizeof(uint32_t), hipHostMallocDefault);
    if (se == hipSuccess) se = hipMalloc((void**)&s.d_data, bytes);
    if (se == hipSuccess) se = hipMalloc((void**)&s.d_offsets, slot_packets * sizeof(uint64_t));
    if (se == hipSuccess) se = hipMalloc((void**)&s.d_lengths, slot_packets * sizeof(uint32_t));
    if (se == hipSuccess) se = hipMalloc((void**)&s.d_crcs, slot_packets * sizeof(uint32_t));
    if (se != hipSuccess) {
      enet_crc_ring_destroy(r);
      return fail_hip(se);
    }
  }
  *out_ring = r;
  return ENET_CRC_OK;
}

void enet_crc_ring_destroy(enet_crc_ring* r) {
  if (!r) return;
  {
    DeviceGuard g(r->device);
    for (auto& s : r->slots) ring_free_slot(s);
  }
  delete r;
}

int enet_crc_ring_slot(enet_crc_ring* r, uint32_t slot, uint8_t** data, uint64_t** offsets, uint32_t** lengths,
                       uint32_t** crcs) {
  if (!r || slot >= r->slots.size()) return ENET_CRC_E_INVALID;
  RingSlot& s = r->slots[slot];
  if (data) *data = s.h_data;
  if (offsets) *offsets = s.h_offsets;
  if (lengths) *lengths = s.h_lengths;
  if (crcs) *crcs = s.h_crcs;
  return ENET_CRC_OK;
}

int enet_crc_ring_submit(enet_crc_ring* r, uint32_t slot, uint64_t count) {
  if (!r || slot >= r->slots.size() || count > r->slot_packets) return ENET_CRC_E_INVALID;
  RingSlot& s = r->slots[slot];
  uint64_t span = 0;  // bytes [0, span) of the slot hold every packet
  for (uint64_t i = 0; i < count; ++i) {
    const uint64_t o = s.h_offsets[i], l = s.h_lengths[i];
    if (o > r->slot_bytes || l > r->slot_bytes - o) return ENET_CRC_E_INVALID;
    span = std::max(span, o + l);
  }
  {
    std::lock_guard<std::mutex> lk(r->lock);
    if (s.busy) return ENET_CRC_E_INVALID;
    s.busy = true;
  }
  DeviceGuard g(r->device);
  auto fail = [&](hipError_t e) {
    std::lock_guard<std::mutex> lk(r->lock);
    s.busy = false;
    return fail_hip(e);
  };
  hipError_t e = hipSuccess;
  if (count) {
    if (span) e = hipMemcpyAsync(s.d_data, s.h_data, span, hipMemcpyHostToDevice, s.stream);
    if (e == hipSuccess)
      e = hipMemcpyAsync(s.d_offsets, s.h_offsets, count * sizeof(uint64_t), hipMemcpyHostToDevice, s.stream);
    if (e == hipSuccess)
      e = hipMemcpyAsync(s.d_lengths, s.h_lengths, count * sizeof(uint32_t), hipMemcpyHostToDevice, s.stream);
    if (e == hipSuccess) e = launch_ragged(s.d_data, s.d_offsets, s.d_lengths, count, s.d_crcs, s.stream);
    if (e == hipSuccess)
      e = hipMemcpyAsync(s.h_crcs, s.d_crcs, count * sizeof(uint32_t), hipMemcpyDeviceToHost, s.stream);
  }
  if (e == hipSuccess) e = hipEventRecord(s.done, s.stream);
  if (e != hipSuccess) return fail(e);
  return ENET_CRC_OK;
}

int enet_crc_ring_wait(enet_crc_ring* r, uint32_t slot) {
  if (!r || slot >= r->slots.size()) return ENET_CRC_E_INVALID;
  RingSlot& s = r->slots[slot];
  {
    std::lock_guard<std::mutex> lk(r->lock);
    if (!s.busy) return ENET_CRC_OK;
  }
  DeviceGuard g(r->device);
  const hipError_t e = hipEventSynchronize(s.done);
  std::lock_guard<std::mutex> lk(r->lock);
  s.busy = false;
  return e == hipSuccess ? ENET_CRC_OK : fail_hip(e);
}

}  // extern "C"

// ---------------------------------------------------------------------------------
// Batched range coder (include/enet_range_amd.h; kernels in range_coder.hip).

static int range_batch(bool decompress, const void* d_in, const uint64_t* d_in_offsets,
                       const uint32_t* d_in_lengths, uint64_t count, void* d_out, const uint64_t* d_out_offsets,
                       const uint32_t* d_out_limits, uint32_t* d_sizes, void* d_scratch, uint64_t scratch_bytes,
                       void* hip_stream) {
  if (count == 0) return ENET_CRC_OK;
  if (!d_in || !d_in_offsets || !d_in_lengths || !d_out || !d_out_offsets || !d_out_limits || !d_sizes ||
      !d_scratch || ((uintptr_t)d_scratch & 15) != 0)
    return ENET_CRC_E_INVALID;
  const uint64_t workers = scratch_bytes / kRangeArenaBytes;
  if (workers == 0) return ENET_CRC_E_INVALID;
  hipError_t e = launch_range(decompress, static_cast<const uint8_t*>(d_in), d_in_offsets, d_in_lengths, count,
                              static_cast<uint8_t*>(d_out), d_out_offsets, d_out_limits, d_sizes, d_scratch, workers,
                              static_cast<hipStream_t>(hip_stream));
  return e == hipSuccess ? ENET_CRC_OK : fail_hip(e);
}

extern "C" {

uint64_t enet_range_scratch_bytes(uint64_t workers) { return workers * kRangeArenaBytes; }

int enet_range_compress_ragged_device(const void* d_in, const uint64_t* d_in_offsets, const uint32_t* d_in_lengths,
                                      uint64_t count, void* d_out, const uint64_t* d_out_offsets,
                                      const uint32_t* d_out_limits, uint32_t* d_sizes, void* d_scratch,
                                      uint64_t scratch_bytes, void* hip_stream) {
  return range_batch(false, d_in, d_in_offsets, d_in_lengths, count, d_out, d_out_offsets, d_out_limits, d_sizes,
                     d_scratch, scratch_bytes, hip_stream);
}

int enet_range_decompress_ragged_device(const void* d_in, const uint64_t* d_in_offsets,
                                        const uint32_t* d_in_lengths, uint64_t count, void* d_out,
                                        const uint64_t* d_out_offsets, const uint32_t* d_out_limits,
                                        uint32_t* d_sizes, void* d_scratch, uint64_t scratch_bytes,
                                        void* hip_stream) {
  return range_batch(true, d_in, d_in_offsets, d_in_lengths, count, d_out, d_out_offsets, d_out_limits, d_sizes,
                     d_scratch, scratch_bytes, hip_stream);
}

}  // extern "C"
