// C ABI of the MI355X CRC-32 path (include/enet_crc_amd.h, include/enet_range_amd.h).
//
// The reference hook is a synchronous `Fn(&[&[u8]]) -> u32` called on the
// thread running Host::service()/flush() (src/host.rs:185-201, src/c/protocol.rs
// :1499 and :2287).  This file maps that surface and the batch entry points
// onto the gfx950 kernels in crc32_kernels.hip / range_coder.hip.  There is no
// CPU path: every checksum comes from the GPU or the call returns an error.
//
// A context owns one "lane" per entry of its device list (duplicates allowed):
// a pair of pinned/device staging slots with their streams, and the range-coder
// staging.  Host-memory batches are split into byte-balanced contiguous shards,
// one per lane; lane 0 runs on the calling thread, the others on the context's
// worker threads (one per extra lane), each on its own device and streams.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <functional>
#include <memory>
#include <mutex>
#include <new>
#include <thread>
#include <vector>

#include "../../include/enet_crc_amd.h"
#include "../../include/enet_range_amd.h"
#include "crc32_host.hpp"
#include "crc32_kernels.hpp"
#include "crc32_mailbox.hpp"
#include "crc32_slot.hpp"
#include "range_coder.hpp"

namespace enet_crc {

namespace {

thread_local int t_last_hip_error = 0;

int fail_hip(hipError_t e) {
  t_last_hip_error = (int)e;
  if (e == hipErrorNoDevice || e == hipErrorInvalidDevice) return ENET_CRC_E_NO_DEVICE;
  if (e == hipErrorOutOfMemory) return ENET_CRC_E_NOMEM;
  return ENET_CRC_E_HIP;
}

#define ENET_HIP_TRY(expr)                     \
  do {                                         \
    hipError_t _e = (expr);                    \
    if (_e != hipSuccess) return fail_hip(_e); \
  } while (0)

#define ENET_TRY(expr)              \
  do {                              \
    int _s = (expr);                \
    if (_s != ENET_CRC_OK) return _s; \
  } while (0)

constexpr int kMaxDevices = 64;
std::atomic<int> g_cu_count[kMaxDevices];
// Restores the caller's current device on scope exit.
struct DeviceGuard {
  int prev = -1;
  explicit DeviceGuard(int dev) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    if (dev >= 0 && prev != dev) (void)hipSetDevice(dev);
  }
  ~DeviceGuard() {
    int cur = -1;
    if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
  }
};

// Device of an explicit stream (-1 for the legacy default stream / an unknown one):
// the device entry points launch on the stream's device, whatever device is current.
int stream_device(hipStream_t s) {
  if (s == nullptr) return -1;
  int d = -1;
  return hipStreamGetDevice(s, &d) == hipSuccess ? d : -1;
}

// The device-side failure channel (crc32_kernels.hpp: FaultWord).  Every slot of a
// synchronous entry (a host-path staging slot, a ring slot) owns a word that only its own
// launches write: the entry clears it before its launches and reads it after its last wait,
// so a failure is reported by the call whose batch failed and by no other.
// The asynchronous *_device entries report into the device's word (enet_crc_device_status).
int slot_fault_word(FaultWord& w) {
  if (w.host) return ENET_CRC_OK;
  const hipError_t e = alloc_fault_word(&w);
  return e == hipSuccess ? ENET_CRC_OK : fail_hip(e);
}
void clear_fault(FaultWord& w) {
  if (w.host) __atomic_store_n(const_cast<uint32_t*>(w.host), 0u, __ATOMIC_RELEASE);
}
bool faulted(const FaultWord& w) {
  return w.host && __atomic_load_n(const_cast<const uint32_t*>(w.host), __ATOMIC_ACQUIRE) != 0u;
}

}  // namespace

// Operator ladder of the slot correction and the flat ragged kernel's finish pass
// (crc32_slot.hpp: kSlotLevels forward + kInvLevels inverse levels + the M8^len(init) table): one host copy, one
// device copy per device (uploaded on first use, never freed: 408 KiB).
std::mutex g_ladder_lock;
uint32_t* g_device_ladder[kMaxDevices];

hipError_t device_slot_ladder(const uint32_t** out) {
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return e;
  if (dev < 0 || dev >= kMaxDevices) return hipErrorInvalidDevice;
  std::lock_guard<std::mutex> lk(g_ladder_lock);
  if (!g_device_ladder[dev]) {
    const size_t bytes = sizeof(uint32_t) * kLadderDwords;
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

// Each device's kick word (ENET_CRC_PERCALL_PERSISTENT).  A resident per-call server wave
// holds a CU, and the batch kernels size their grids to one workgroup per CU with a static
// share each: measured next to an answering server, a G2-shaped batch took 141-149 us
// instead of ~88 (profiles/r03/s3, s4/server_latency.txt) -- one workgroup waited for a
// whole share -- and holding CUs back for it instead cost 6-10 % (server_overlap.txt).  So
// the first workgroup of every batch kernel bumps the word as it starts
// (send_servers_home, crc32_kernels.hip); a server exits as soon as it reads another value
// than at its start, and the next per-call call relaunches it.
std::atomic<uint32_t*> g_kick_dev[kMaxDevices];  // device address of the word
std::mutex g_kick_lock;

// The kick word of `dev` (allocated on first use: fine-grained device memory, or mapped
// pinned host memory when the device's memory is not host-visible), registered with the
// batch kernels of that device.
hipError_t kick_word(int dev, uint32_t** dev_ptr) {
  if (!g_kick_dev[dev].load(std::memory_order_acquire)) {
    std::lock_guard<std::mutex> lk(g_kick_lock);
    if (!g_kick_dev[dev].load(std::memory_order_relaxed)) {
      DeviceGuard g(dev);
      uint32_t* d = nullptr;
      if (hipExtMallocWithFlags((void**)&d, 128, hipDeviceMallocFinegrained) == hipSuccess) {
        hipError_t e = hipMemset(d, 0, 128);
        if (e != hipSuccess) return e;
      } else {
        (void)hipGetLastError();
        uint32_t* h = nullptr;
        hipError_t e = hipHostMalloc((void**)&h, 128, hipHostMallocMapped | hipHostMallocCoherent);
        if (e != hipSuccess) return e;
        memset(h, 0, 128);
        e = hipHostGetDevicePointer((void**)&d, h, 0);
        if (e != hipSuccess) return e;
      }
      const hipError_t e = set_device_kick_word(d);
      if (e != hipSuccess) return e;
      g_kick_dev[dev].store(d, std::memory_order_release);
    }
  }
  *dev_ptr = g_kick_dev[dev].load(std::memory_order_acquire);
  return hipSuccess;
}

// CUs a batch launch on the current device sizes its grid to: all of them (a resident
// per-call server is sent home by the kernel itself, see g_kick_dev).
int cu_count_for_current_device() {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kMaxDevices) return -1;
  int n = g_cu_count[dev].load(std::memory_order_relaxed);
  if (n <= 0) {
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return -1;
    g_cu_count[dev].store(n, std::memory_order_relaxed);
  }
#ifdef ENET_CRC_TEST_HOOKS
  // Test build only: ENET_CRC_TEST_RESERVE=n holds back n CUs (scripts/exp_server_overlap.py).
  constexpr int kXcds = 8;
  if (const char* v = getenv("ENET_CRC_TEST_RESERVE")) {
    const int reserve = atoi(v);
    return n - reserve >= kXcds ? n - reserve : kXcds;
  }
#endif
  return n;
}


}  // namespace enet_crc

using namespace enet_crc;

namespace {

// Pinned host buffer + device mirror of `T`, grown on demand (contents not kept).
template <typename T>
struct Mirror {
  T* h = nullptr;
  T* d = nullptr;
  size_t cap = 0;  // elements
  int grow(size_t n, size_t pad_bytes = 0) {
    if (n <= cap && h) return ENET_CRC_OK;
    release();
    n = std::max<size_t>(n, 64);
    const size_t bytes = (n * sizeof(T) + pad_bytes + 15) & ~(size_t)15;
    ENET_HIP_TRY(hipHostMalloc((void**)&h, bytes, hipHostMallocDefault));
    ENET_HIP_TRY(hipMalloc((void**)&d, bytes));
    cap = n;
    return ENET_CRC_OK;
  }
  void release() {
    if (h) (void)hipHostFree(h);
    if (d) (void)hipFree(d);
    h = nullptr;
    d = nullptr;
    cap = 0;
  }
};

// One pipeline slot of the host path: pinned input bytes + descriptors, device
// copies, pinned output.
struct StageSlot {
  Mirror<uint8_t> bytes;  // +16 B: the kernels' 4-byte-grid loads stay inside whole 16-B lines
  Mirror<uint64_t> offsets;
  Mirror<uint32_t> lengths;
  Mirror<uint32_t> out;
  hipStream_t stream = nullptr;
  hipEvent_t done = nullptr;
  FaultWord fault;     // failure word of this slot's ragged launches
  uint64_t first = 0;  // packet range staged in this slot
  uint64_t n = 0;
  bool busy = false;
  void release() {
    bytes.release();
    offsets.release();
    lengths.release();
    out.release();
  }
};

// Range-coder staging of a lane (host-memory compress/decompress entry points).
struct RangeStage {
  Mirror<uint8_t> in, out;
  Mirror<uint64_t> in_off, out_off;
  Mirror<uint32_t> in_len, out_lim, sizes;
  void* d_scratch = nullptr;
  uint64_t workers = 0;
  void release() {
    in.release();
    out.release();
    in_off.release();
    out_off.release();
    in_len.release();
    out_lim.release();
    sizes.release();
    if (d_scratch) (void)hipFree(d_scratch);
    d_scratch = nullptr;
    workers = 0;
  }
};

// Per-call (enet_crc32_iov) buffers: a pinned, device-mapped input buffer the kernel
// reads directly (zero-copy mode), a mapped result word, and the persistent server's
// mailbox (pinned, coherent, mapped) with its stream.
struct PerCall {
  uint8_t* h_in = nullptr;
  size_t cap = 0;
  uint32_t* h_res = nullptr;  // [0] = checksum (mapped: written by the kernel)
  Mailbox* mb = nullptr;      // host address of the answer mailbox (pinned host memory)
  Mailbox* d_mb = nullptr;    // its device address
  Mailbox* req = nullptr;     // host address of the request mailbox
  Mailbox* d_req = nullptr;   // its device address
  bool req_vram = false;      // request mailbox in device memory written through the BAR
  hipStream_t mb_stream = nullptr;
  int mb_device = 0;          // device of mb_stream (lane 0's)
  bool mb_launched = false;   // a server was launched and may still run
  bool mb_wedged = false;     // a stop request was not honoured within kServerStopLimit
  uint32_t mb_seq = 0;        // last request number posted
};

// The only writer of PerCall::mb_launched.
void set_server_live(PerCall& c, bool live) { c.mb_launched = live; }

// A worker thread bound to one lane: runs one job at a time for the calling thread.
class Worker {
 public:
  Worker() : th_([this] { loop(); }) {}
  ~Worker() {
    {
      std::lock_guard<std::mutex> g(m_);
      quit_ = true;
    }
    cv_.notify_all();
    th_.join();
  }
  void start(std::function<int()> job) {
    {
      std::lock_guard<std::mutex> g(m_);
      job_ = std::move(job);
      has_job_ = true;
      done_ = false;
    }
    cv_.notify_all();
  }
  int wait() {
    std::unique_lock<std::mutex> g(m_);
    cv_.wait(g, [this] { return done_; });
    return result_;
  }

 private:
  void loop() {
    std::unique_lock<std::mutex> g(m_);
    for (;;) {
      cv_.wait(g, [this] { return has_job_ || quit_; });
      if (quit_) return;
      std::function<int()> job = std::move(job_);
      has_job_ = false;
      g.unlock();
      const int r = job();
      g.lock();
      result_ = r;
      done_ = true;
      cv_.notify_all();
    }
  }
  std::mutex m_;
  std::condition_variable cv_;
  std::function<int()> job_;
  bool has_job_ = false, done_ = true, quit_ = false;
  int result_ = ENET_CRC_OK;
  std::thread th_;
};

struct Lane {
  int device = 0;
  StageSlot slot[2];
  RangeStage range;
  std::unique_ptr<Worker> worker;  // lanes >= 1
};

}  // namespace

struct enet_crc_ctx {
  std::mutex lock;
  std::vector<Lane> lanes;
  PerCall call;
  int percall_mode = ENET_CRC_PERCALL_ZEROCOPY;
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
  FaultWord fault;  // failure word of this slot's launches (cleared by submit, read by wait)
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

// A persistent-mode call gives up on the server after this long (test build: 200 ms), and
// a stop request waits at most kServerStopLimit for the server's stream to drain (longer
// than the server's 2-s lifetime, so only a wedged wave misses it; test build: 100 ms).
#ifdef ENET_CRC_TEST_HOOKS
constexpr std::chrono::milliseconds kMailboxCallTimeout(200);
constexpr std::chrono::milliseconds kServerStopLimit(100);
#else
constexpr std::chrono::milliseconds kMailboxCallTimeout(5000);
constexpr std::chrono::milliseconds kServerStopLimit(3000);
#endif

// Host path chunking: at most this many staged bytes / packets per slot.
constexpr size_t kStageBytes = 64u << 20;
constexpr size_t kStagePackets = 1u << 18;
// Concurrent coders of a host-memory range-coder batch (scratch: workers x 64 KiB).
constexpr uint64_t kRangeHostWorkers = 16384;

#ifdef ENET_CRC_TEST_HOOKS
// Test build only (make testhooks; tests/test_gpu_hooks.py): the k-th chunk (1-based) of
// every enet_crc32_ragged_host shard fails as if its staging allocation had.
int injected_stage_fault() {
  const char* v = getenv("ENET_CRC_TEST_STAGE_FAULT");
  return v ? atoi(v) : 0;
}
#else
constexpr int injected_stage_fault() { return 0; }
#endif

// Waits for whatever the lane's slots still have in flight and forgets it (error exits:
// no copy-out into the caller's buffers, no buffer reuse under a running copy).
void quiesce(Lane& L) {
  for (auto& s : L.slot) {
    if (s.busy && s.stream) (void)hipStreamSynchronize(s.stream);
    s.busy = false;
  }
}

// Packets [0, count) of one shard, on lane L's device: chunks of <= 64 MiB / 256K
// packets alternate between the two staging slots, so the H2D copy of chunk i+1
// overlaps the kernel of chunk i.  Caller holds the context lock.
int ragged_host_shard(Lane& L, const uint8_t* base, const uint64_t* h_offsets, const uint32_t* h_lengths,
                      uint64_t count, uint32_t* h_out) {
  if (count == 0) return ENET_CRC_OK;
  DeviceGuard g(L.device);
  struct Quiesce {
    Lane& L;
    bool armed = true;
    ~Quiesce() {
      if (armed) quiesce(L);
    }
  } guard{L};
  const int fault_at = injected_stage_fault();
  for (auto& s : L.slot) {
    ENET_TRY(slot_fault_word(s.fault));
    clear_fault(s.fault);  // both slots are idle here (quiesced by any earlier exit)
  }

  // Drain a slot: wait for its kernel + D2H, copy checksums out.
  auto drain = [&](StageSlot& s) -> int {
    if (!s.busy) return ENET_CRC_OK;
    ENET_HIP_TRY(hipEventSynchronize(s.done));
    memcpy(h_out + s.first, s.out.h, s.n * sizeof(uint32_t));
    s.busy = false;
    return ENET_CRC_OK;
  };

  uint64_t p = 0;
  int which = 0, chunk = 0;
  while (p < count) {
    StageSlot& s = L.slot[which];
    ENET_TRY(drain(s));
    const StageChunk ch = plan_stage_chunk(h_offsets, h_lengths, count, p, kStageBytes, kStagePackets);
    if (++chunk == fault_at) return ENET_CRC_E_NOMEM;
    const uint64_t q = ch.end, lo_al = ch.lo_al;
    const size_t span = (size_t)ch.span;
    const size_t n = (size_t)(q - p);
    ENET_TRY(s.bytes.grow(std::max<size_t>(span, 4096), 16));
    ENET_TRY(s.offsets.grow(n));
    ENET_TRY(s.lengths.grow(n));
    ENET_TRY(s.out.grow(n));
    memcpy(s.bytes.h, base + lo_al, span);
    for (uint64_t i = p; i < q; ++i) {
      s.offsets.h[i - p] = h_offsets[i] - lo_al;
      s.lengths.h[i - p] = h_lengths[i];
    }
    s.first = p;
    s.n = n;
    s.busy = true;  // from here on the slot's stream may hold work: quiesce() waits for it
    ENET_HIP_TRY(hipMemcpyAsync(s.bytes.d, s.bytes.h, span, hipMemcpyHostToDevice, s.stream));
    ENET_HIP_TRY(hipMemcpyAsync(s.offsets.d, s.offsets.h, n * sizeof(uint64_t), hipMemcpyHostToDevice, s.stream));
    ENET_HIP_TRY(hipMemcpyAsync(s.lengths.d, s.lengths.h, n * sizeof(uint32_t), hipMemcpyHostToDevice, s.stream));
    ENET_HIP_TRY(launch_ragged(s.bytes.d, s.offsets.d, s.lengths.d, n, s.out.d, s.stream, s.fault.dev));
    ENET_HIP_TRY(hipMemcpyAsync(s.out.h, s.out.d, n * sizeof(uint32_t), hipMemcpyDeviceToHost, s.stream));
    ENET_HIP_TRY(hipEventRecord(s.done, s.stream));
    p = q;
    which ^= 1;
  }
  for (auto& s : L.slot) ENET_TRY(drain(s));
  guard.armed = false;
  for (auto& s : L.slot)
    if (faulted(s.fault)) return ENET_CRC_E_DEVICE;
  return ENET_CRC_OK;
}

void destroy_lane(Lane& L) {
  L.worker.reset();  // joins the thread first: no job can still be using the buffers
  DeviceGuard g(L.device);
  for (auto& s : L.slot) {
    if (s.stream) (void)hipStreamSynchronize(s.stream);
    s.release();
    if (s.done) (void)hipEventDestroy(s.done);
    if (s.stream) (void)hipStreamDestroy(s.stream);
    free_fault_word(s.fault);
    s.stream = nullptr;
    s.done = nullptr;
  }
  L.range.release();
}

// Runs job(lane index) on every lane: lane 0 on this thread, the others on their
// workers; returns the first non-OK status (all lanes have finished by then).
int run_on_lanes(enet_crc_ctx* ctx, uint32_t nlanes, const std::function<int(uint32_t)>& job) {
  for (uint32_t i = 1; i < nlanes; ++i) ctx->lanes[i].worker->start([&job, i] { return job(i); });
  int st = job(0);
  for (uint32_t i = 1; i < nlanes; ++i) {
    const int r = ctx->lanes[i].worker->wait();
    if (st == ENET_CRC_OK) st = r;
  }
  return st;
}

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
    case ENET_CRC_E_DEVICE: return "a batch kernel gave up on the device (outputs invalid)";
    default: return "unknown status";
  }
}

int enet_crc_last_hip_error(void) { return t_last_hip_error; }

int enet_crc_device_status(int device, int clear) {
  int n = 0;
  const hipError_t e = hipGetDeviceCount(&n);
  if (e != hipSuccess || n <= 0) return e == hipSuccess || e == hipErrorNoDevice ? ENET_CRC_E_NO_DEVICE : fail_hip(e);
  if (device < 0 || device >= n) return ENET_CRC_E_NO_DEVICE;
  FaultWord w;
  const hipError_t fe = device_fault_word(device, &w);
  if (fe != hipSuccess) return fail_hip(fe);
  uint32_t* const h = const_cast<uint32_t*>(w.host);
  const uint32_t v = clear ? __atomic_exchange_n(h, 0u, __ATOMIC_ACQ_REL) : __atomic_load_n(h, __ATOMIC_ACQUIRE);
  return (int)(v & 0x7FFFFFFFu);
}

int enet_crc_device_count(void) {
  int n = 0;
  hipError_t e = hipGetDeviceCount(&n);
  if (e == hipErrorNoDevice) return 0;
  if (e != hipSuccess) return fail_hip(e);
  return n;
}

int enet_crc_shard_bounds(const uint32_t* lengths, uint64_t count, uint32_t nshards, uint64_t* bounds) {
  if (nshards == 0 || !bounds) return ENET_CRC_E_INVALID;
  split_bounds(lengths, count, nshards, bounds);
  return ENET_CRC_OK;
}

int enet_crc_ctx_create_multi(const int* devices, uint32_t ndevices, enet_crc_ctx** out_ctx) {
  if (!out_ctx) return ENET_CRC_E_INVALID;
  *out_ctx = nullptr;
  if (!devices || ndevices == 0 || ndevices > ENET_CRC_MAX_LANES) return ENET_CRC_E_INVALID;
  int n = 0;
  hipError_t e = hipGetDeviceCount(&n);
  if (e != hipSuccess || n <= 0) return e == hipSuccess || e == hipErrorNoDevice ? ENET_CRC_E_NO_DEVICE : fail_hip(e);
  for (uint32_t i = 0; i < ndevices; ++i)
    if (devices[i] < 0 || devices[i] >= n) return ENET_CRC_E_NO_DEVICE;
  enet_crc_ctx* ctx = new (std::nothrow) enet_crc_ctx();
  if (!ctx) return ENET_CRC_E_NOMEM;
  ctx->lanes.resize(ndevices);
  for (uint32_t i = 0; i < ndevices; ++i) {
    Lane& L = ctx->lanes[i];
    L.device = devices[i];
    DeviceGuard g(L.device);
    for (auto& s : L.slot) {
      hipError_t se = hipStreamCreateWithFlags(&s.stream, hipStreamNonBlocking);
      if (se == hipSuccess) se = hipEventCreateWithFlags(&s.done, hipEventDisableTiming);
      if (se != hipSuccess) {
        enet_crc_ctx_destroy(ctx);
        return fail_hip(se);
      }
    }
    if (i > 0) L.worker.reset(new (std::nothrow) Worker());
    if (i > 0 && !L.worker) {
      enet_crc_ctx_destroy(ctx);
      return ENET_CRC_E_NOMEM;
    }
  }
  *out_ctx = ctx;
  return ENET_CRC_OK;
}

int enet_crc_ctx_create(int device, enet_crc_ctx** out_ctx) { return enet_crc_ctx_create_multi(&device, 1, out_ctx); }

int enet_crc_ctx_lanes(const enet_crc_ctx* ctx) { return ctx ? (int)ctx->lanes.size() : ENET_CRC_E_INVALID; }

namespace {

// Ask a running server to exit and wait for its stream at most `limit`.  Returns whether
// it drained; if not, the wave stays counted as resident and is marked wedged: later stops
// only re-check it (no second wait), persistent calls fail at once, and destroy leaks the
// stream and mailbox memory the wave may still touch instead of hanging on it.
bool stop_mailbox_bounded(PerCall& c, std::chrono::milliseconds limit) {
  if (!c.mb_launched) return true;
  if (c.mb_wedged) limit = std::chrono::milliseconds(0);
  __atomic_store_n(&c.req->seq, kMailboxStop, __ATOMIC_RELEASE);
  __builtin_ia32_sfence();
  const auto t0 = std::chrono::steady_clock::now();
  while (hipStreamQuery(c.mb_stream) == hipErrorNotReady) {
    if (std::chrono::steady_clock::now() - t0 >= limit) {
      c.mb_wedged = true;
      return false;
    }
    std::this_thread::sleep_for(std::chrono::microseconds(100));
  }
  set_server_live(c, false);
  c.mb_wedged = false;
  return true;
}

// Ask a running server to exit and wait until it has (bounded by kServerStopLimit).
void stop_mailbox(PerCall& c) { (void)stop_mailbox_bounded(c, kServerStopLimit); }

}  // namespace

// Batch entry points of a context stop its server wave first: a resident wave holds
// one CU, and the batched kernels size their grids to every CU.  False when the wave did
// not stop within kServerStopLimit (wedged): the batch still runs, its workgroup on that CU
// starting once the wave ends (at its 2-s lifetime); enet_crc_ctx_stop_server reports it.
static bool stop_server_for_batch(enet_crc_ctx* ctx) {
  if (!ctx->call.mb_launched) return true;
  DeviceGuard g(ctx->lanes[0].device);
  return stop_mailbox_bounded(ctx->call, kServerStopLimit);
}

int enet_crc_ctx_set_percall_mode(enet_crc_ctx* ctx, int mode) {
  if (!ctx || (mode != ENET_CRC_PERCALL_COPY && mode != ENET_CRC_PERCALL_ZEROCOPY &&
               mode != ENET_CRC_PERCALL_PERSISTENT))
    return ENET_CRC_E_INVALID;
  std::lock_guard<std::mutex> lk(ctx->lock);
  if (mode != ENET_CRC_PERCALL_PERSISTENT && ctx->call.mb_launched) {
    DeviceGuard g(ctx->lanes[0].device);
    stop_mailbox(ctx->call);
  }
  ctx->percall_mode = mode;
  return ENET_CRC_OK;
}

int enet_crc_ctx_percall_mode(enet_crc_ctx* ctx) {
  if (!ctx) return ENET_CRC_E_INVALID;
  std::lock_guard<std::mutex> lk(ctx->lock);
  return ctx->percall_mode;
}

int enet_crc_ctx_stop_server(enet_crc_ctx* ctx) {
  if (!ctx) return ENET_CRC_E_INVALID;
  std::lock_guard<std::mutex> lk(ctx->lock);
  // A wave that ignores the stop request: say so instead of returning OK while
  // it still holds a CU.
  return stop_server_for_batch(ctx) ? ENET_CRC_OK : fail_hip(hipErrorLaunchTimeOut);
}

void enet_crc_ctx_destroy(enet_crc_ctx* ctx) {
  if (!ctx) return;
  if (!ctx->lanes.empty()) {
    DeviceGuard g(ctx->lanes[0].device);
    stop_mailbox(ctx->call);
  }
  if (ctx->call.mb_launched) {
    // The server wave ignored the stop request (mb_wedged).  Every free below would wait
    // for the device, i.e. for that wave: leak the context's device and pinned memory and
    // its streams instead of hanging (the worker threads are still joined).
    for (auto& L : ctx->lanes) L.worker.reset();
    delete ctx;
    return;
  }
  for (auto& L : ctx->lanes) destroy_lane(L);
  if (!ctx->lanes.empty()) {
    DeviceGuard g(ctx->lanes[0].device);
    if (ctx->call.h_in) (void)hipHostFree(ctx->call.h_in);
    if (ctx->call.h_res) (void)hipHostFree(ctx->call.h_res);
    if (ctx->call.req && ctx->call.req_vram) (void)hipFree(ctx->call.d_req);
    if (ctx->call.mb) (void)hipHostFree(ctx->call.mb);
    if (ctx->call.mb_stream) (void)hipStreamDestroy(ctx->call.mb_stream);
  }
  delete ctx;
}

int enet_crc32_uniform_device(const void* d_base, uint64_t stride, uint32_t length, uint64_t count,
                              uint32_t* d_out, void* hip_stream) {
  if (count == 0) return ENET_CRC_OK;
  if (!d_out || (!d_base && length > 0)) return ENET_CRC_E_INVALID;
  const hipStream_t stream = static_cast<hipStream_t>(hip_stream);
  DeviceGuard g(stream_device(stream));
  hipError_t e = launch_uniform(static_cast<const uint8_t*>(d_base), stride, length, count, d_out, stream);
  return e == hipSuccess ? ENET_CRC_OK : fail_hip(e);
}

int enet_crc32_ragged_device(const void* d_base, const uint64_t* d_offsets, const uint32_t* d_lengths,
                             uint64_t count, uint32_t* d_out, void* hip_stream) {
  if (count == 0) return ENET_CRC_OK;
  if (!d_base || !d_offsets || !d_lengths || !d_out) return ENET_CRC_E_INVALID;
  const hipStream_t stream = static_cast<hipStream_t>(hip_stream);
  DeviceGuard g(stream_device(stream));
  hipError_t e = launch_ragged(static_cast<const uint8_t*>(d_base), d_offsets, d_lengths, count, d_out, stream);
  return e == hipSuccess ? ENET_CRC_OK : fail_hip(e);
}

namespace {

// Whether `p` is device memory of device `dev` (any address inside a hipMalloc'd block).
bool on_device(const void* p, int dev) {
  hipPointerAttribute_t a;
  if (hipPointerGetAttributes(&a, p) != hipSuccess) {
    (void)hipGetLastError();  // an unregistered host pointer: not device memory
    return false;
  }
  return a.type == hipMemoryTypeDevice && a.device == dev;
}

}  // namespace

int enet_crc32_shards_device(const enet_crc_shard* shards, size_t nshards) {
  if (nshards > 0 && !shards) return ENET_CRC_E_INVALID;
  int ndev = 0;
  if (nshards > 0) {
    const hipError_t e = hipGetDeviceCount(&ndev);
    if (e != hipSuccess || ndev <= 0) return e == hipSuccess || e == hipErrorNoDevice ? ENET_CRC_E_NO_DEVICE : fail_hip(e);
  }
  // Placement is checked for every shard before anything launches: each shard's buffers
  // and stream must belong to its own device (a misplaced shard would otherwise run as
  // peer reads across the fabric, or fault).
  for (size_t i = 0; i < nshards; ++i) {
    const enet_crc_shard& s = shards[i];
    if (s.count == 0) continue;
    if (!s.d_out || !s.d_base || (s.d_offsets != nullptr) != (s.d_lengths != nullptr)) return ENET_CRC_E_INVALID;
    if (s.device < 0 || s.device >= ndev) return ENET_CRC_E_NO_DEVICE;
    if (!on_device(s.d_base, s.device) || !on_device(s.d_out, s.device) ||
        (s.d_offsets && (!on_device(s.d_offsets, s.device) || !on_device(s.d_lengths, s.device))))
      return ENET_CRC_E_INVALID;
    if (s.hip_stream && stream_device(static_cast<hipStream_t>(s.hip_stream)) != s.device) return ENET_CRC_E_INVALID;
  }
  for (size_t i = 0; i < nshards; ++i) {
    const enet_crc_shard& s = shards[i];
    if (s.count == 0) continue;
    DeviceGuard g(s.device);
    const hipStream_t stream = static_cast<hipStream_t>(s.hip_stream);
    const uint8_t* base = static_cast<const uint8_t*>(s.d_base);
    const hipError_t e = s.d_offsets ? launch_ragged(base, s.d_offsets, s.d_lengths, s.count, s.d_out, stream)
                                     : launch_uniform(base, s.stride, s.length, s.count, s.d_out, stream);
    if (e != hipSuccess) return fail_hip(e);
  }
  return ENET_CRC_OK;
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
  DeviceGuard g(stream_device(stream));
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
  return slot_adjust_checksum(crc, old_slot, new_slot, bytes_after_slot);
}

uint32_t enet_crc32_combine(uint32_t crc_a, uint32_t crc_b, uint64_t len_b) {
  return combine_checksums(crc_a, crc_b, len_b);
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
  Lane& L = ctx->lanes[0];
  DeviceGuard g(L.device);
  StageSlot& s = L.slot[0];
  quiesce(L);  // nothing of an earlier (failed) call may still use the buffers
  if (ctx->percall_mode == ENET_CRC_PERCALL_PERSISTENT && total <= kMailboxBytes) {
    // Post the datagram to the server wave's mailbox and spin on its answer; launch the
    // server when none runs (first call, or it exited after kMailboxIdleTicks idle).
    PerCall& c = ctx->call;
    if (!c.mb) {
      ENET_HIP_TRY(hipHostMalloc((void**)&c.mb, sizeof(Mailbox), hipHostMallocMapped | hipHostMallocCoherent));
      memset(c.mb, 0, sizeof(Mailbox));
      ENET_HIP_TRY(hipHostGetDevicePointer((void**)&c.d_mb, c.mb, 0));
      ENET_HIP_TRY(hipStreamCreateWithFlags(&c.mb_stream, hipStreamNonBlocking));
      c.mb_device = L.device;
      // Requests: in fine-grained device memory that the host writes through the PCIe BAR
      // when the whole VRAM is host-visible (large BAR), so the server reads each
      // datagram locally instead of across PCIe; otherwise the answer
      // mailbox doubles as the request mailbox.
      int large_bar = 0;
      if (hipDeviceGetAttribute(&large_bar, hipDeviceAttributeIsLargeBar, L.device) == hipSuccess && large_bar &&
          hipExtMallocWithFlags((void**)&c.d_req, sizeof(Mailbox), hipDeviceMallocFinegrained) == hipSuccess) {
        c.req = c.d_req;  // one address for host and device
        c.req_vram = true;
        memset(c.req, 0, sizeof(Mailbox));
        __builtin_ia32_sfence();
      } else {
        (void)hipGetLastError();
        c.req = c.mb;
        c.d_req = c.d_mb;
      }
    }
    // A server that ignored a stop request still owns the mailbox: fail at once (until
    // its stream drains) rather than post into it and wait for the call time-out.
    if (c.mb_wedged && !stop_mailbox_bounded(c, std::chrono::milliseconds(0))) return fail_hip(hipErrorLaunchTimeOut);
    const uint32_t* ladder = nullptr;
    ENET_HIP_TRY(device_slot_ladder(&ladder));
    uint8_t* dst = c.req->data + (kMailboxBytes - total);  // right-aligned; zero below it in its chunk
    memset(c.req->data + ((kMailboxBytes - total) & ~(size_t)63), 0, (kMailboxBytes - total) & 63);
    size_t pos = 0;  // concatenation, src/crc32.rs:41-42
    for (size_t i = 0; i < nbufs; ++i) {
      if (bufs[i].len) memcpy(dst + pos, bufs[i].data, bufs[i].len);
      pos += bufs[i].len;
    }
    c.mb_seq = c.mb_seq + 1 == kMailboxStop ? 1u : c.mb_seq + 1;
    const uint32_t seq = c.mb_seq;
    // seq and len in one 64-bit store, ordered after the bytes.  Through the BAR the
    // mapping is write-combining: sfence drains the bytes before the store and the store
    // itself right after it (without it a store can sit in the buffer for milliseconds).
    if (c.req_vram) __builtin_ia32_sfence();
    __atomic_store_n(reinterpret_cast<uint64_t*>(&c.req->seq), ((uint64_t)total << 32) | seq, __ATOMIC_RELEASE);
    if (c.req_vram) __builtin_ia32_sfence();
    uint32_t* kick = nullptr;
    ENET_HIP_TRY(kick_word(c.mb_device, &kick));
    auto launch = [&]() -> hipError_t {
      const hipError_t e = launch_mailbox(c.d_req, c.d_mb, ladder, kick, c.mb_stream);
      set_server_live(c, e == hipSuccess);
      return e;
    };
    if (!c.mb_launched || hipStreamQuery(c.mb_stream) == hipSuccess) ENET_HIP_TRY(launch());
    const auto t0 = std::chrono::steady_clock::now();
    const uint64_t* answer = reinterpret_cast<const uint64_t*>(&c.mb->done);  // done | result << 32
    uint64_t a = 0;
    for (uint32_t n = 1; (uint32_t)(a = __atomic_load_n(answer, __ATOMIC_ACQUIRE)) != seq; ++n) {
      if ((n & 1023u) == 0) {
        // The server may have exited (idle limit) just before this request: relaunch.
        if (hipStreamQuery(c.mb_stream) == hipSuccess && (uint32_t)__atomic_load_n(answer, __ATOMIC_ACQUIRE) != seq)
          ENET_HIP_TRY(launch());
        if (std::chrono::steady_clock::now() - t0 > kMailboxCallTimeout) {
          // No answer: stop the server (bounded wait) and leave persistent mode for good
          // on this context, so later calls do not wait for a wedged wave again; the
          // caller may select persistent mode once more (enet_crc_ctx_set_percall_mode).
          (void)stop_mailbox_bounded(c, std::chrono::milliseconds(100));
          ctx->percall_mode = ENET_CRC_PERCALL_ZEROCOPY;
          return fail_hip(hipErrorLaunchTimeOut);
        }
      }
      __builtin_ia32_pause();
    }
    const uint32_t reg = (uint32_t)(a >> 32) ^ host_slot_ladder()[kLadderLevels * kSlotLevelDwords + total];
    *out_crc = __builtin_bswap32(~reg);
    return ENET_CRC_OK;
  }
  if (ctx->percall_mode != ENET_CRC_PERCALL_COPY) {
    // The kernel reads the gathered bytes straight from pinned host memory and writes
    // the checksum into mapped host memory: no copy engine on the path.
    PerCall& c = ctx->call;
    if (total + 16 > c.cap || !c.h_in) {
      if (c.h_in) (void)hipHostFree(c.h_in);
      c.h_in = nullptr;
      c.cap = 0;
      const size_t cap = std::max<size_t>((total + 16 + 4095) & ~(size_t)4095, 8192);
      ENET_HIP_TRY(hipHostMalloc((void**)&c.h_in, cap, hipHostMallocMapped));
      c.cap = cap;
    }
    if (!c.h_res) ENET_HIP_TRY(hipHostMalloc((void**)&c.h_res, 64, hipHostMallocMapped | hipHostMallocCoherent));
    size_t pos = 0;  // concatenation, src/crc32.rs:41-42
    for (size_t i = 0; i < nbufs; ++i) {
      if (bufs[i].len) memcpy(c.h_in + pos, bufs[i].data, bufs[i].len);
      pos += bufs[i].len;
    }
    uint8_t* d_in = nullptr;
    uint32_t* d_res = nullptr;
    ENET_HIP_TRY(hipHostGetDevicePointer((void**)&d_in, c.h_in, 0));
    ENET_HIP_TRY(hipHostGetDevicePointer((void**)&d_res, c.h_res, 0));
    ENET_HIP_TRY(launch_single(d_in, (uint32_t)total, d_res, s.stream));
    ENET_HIP_TRY(hipStreamSynchronize(s.stream));
    *out_crc = __atomic_load_n(&c.h_res[0], __ATOMIC_ACQUIRE);
    return ENET_CRC_OK;
  }
  ENET_TRY(s.bytes.grow(std::max<size_t>(total, 4096), 16));
  ENET_TRY(s.out.grow(1));
  size_t pos = 0;  // concatenation, src/crc32.rs:41-42
  for (size_t i = 0; i < nbufs; ++i) {
    if (bufs[i].len) memcpy(s.bytes.h + pos, bufs[i].data, bufs[i].len);
    pos += bufs[i].len;
  }
  s.busy = true;
  if (total) ENET_HIP_TRY(hipMemcpyAsync(s.bytes.d, s.bytes.h, total, hipMemcpyHostToDevice, s.stream));
  ENET_HIP_TRY(launch_uniform(s.bytes.d, 0, (uint32_t)total, 1, s.out.d, s.stream));
  ENET_HIP_TRY(hipMemcpyAsync(s.out.h, s.out.d, sizeof(uint32_t), hipMemcpyDeviceToHost, s.stream));
  ENET_HIP_TRY(hipStreamSynchronize(s.stream));
  s.busy = false;
  *out_crc = s.out.h[0];
  return ENET_CRC_OK;
}

int enet_crc32_ragged_host(enet_crc_ctx* ctx, const void* h_base, const uint64_t* h_offsets,
                           const uint32_t* h_lengths, uint64_t count, uint32_t* h_out) {
  if (!ctx) return ENET_CRC_E_INVALID;
  if (count == 0) return ENET_CRC_OK;
  if (!h_base || !h_offsets || !h_lengths || !h_out) return ENET_CRC_E_INVALID;
  std::lock_guard<std::mutex> lk(ctx->lock);
  (void)stop_server_for_batch(ctx);  // a wedged wave only delays one workgroup
  const uint8_t* base = static_cast<const uint8_t*>(h_base);
  const uint32_t nl = (uint32_t)std::min<uint64_t>(ctx->lanes.size(), count);
  if (nl <= 1) return ragged_host_shard(ctx->lanes[0], base, h_offsets, h_lengths, count, h_out);
  std::vector<uint64_t> b(nl + 1);
  split_bounds(h_lengths, count, nl, b.data());
  return run_on_lanes(ctx, nl, [&](uint32_t i) {
    return ragged_host_shard(ctx->lanes[i], base, h_offsets + b[i], h_lengths + b[i], b[i + 1] - b[i], h_out + b[i]);
  });
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
  free_fault_word(s.fault);
  s = RingSlot{};
}

int enet_crc_ring_create(int device, uint32_t nslots, uint64_t slot_bytes, uint32_t slot_packets,
                         enet_crc_ring** out_ring) {
  if (!out_ring) return ENET_CRC_E_INVALID;
  *out_ring = nullptr;
  if (nslots == 0 || nslots > 64 || slot_bytes == 0 || slot_packets == 0) return ENET_CRC_E_INVALID;
  int n = 0;
  hipError_t e = hipGetDeviceCount(&n);
  if (e != hipSuccess || n <= 0) return e == hipSuccess || e == hipErrorNoDevice ? ENET_CRC_E_NO_DEVICE : fail_hip(e);
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
    if (se == hipSuccess) se = alloc_fault_word(&s.fault);
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
  {
    std::lock_guard<std::mutex> lk(r->lock);
    if (s.busy) return ENET_CRC_E_INVALID;
    s.busy = true;
  }
  uint64_t span = 0;  // bytes [0, span) of the slot hold every packet
  for (uint64_t i = 0; i < count; ++i) {
    const uint64_t o = s.h_offsets[i], l = s.h_lengths[i];
    if (o > r->slot_bytes || l > r->slot_bytes - o) {
      std::lock_guard<std::mutex> lk(r->lock);
      s.busy = false;
      return ENET_CRC_E_INVALID;
    }
    span = std::max(span, o + l);
  }
  DeviceGuard g(r->device);
  clear_fault(s.fault);  // the slot is idle (not busy): nothing of its own writes the word
  hipError_t e = hipSuccess;
  if (count) {
    if (span) e = hipMemcpyAsync(s.d_data, s.h_data, span, hipMemcpyHostToDevice, s.stream);
    if (e == hipSuccess)
      e = hipMemcpyAsync(s.d_offsets, s.h_offsets, count * sizeof(uint64_t), hipMemcpyHostToDevice, s.stream);
    if (e == hipSuccess)
      e = hipMemcpyAsync(s.d_lengths, s.h_lengths, count * sizeof(uint32_t), hipMemcpyHostToDevice, s.stream);
    if (e == hipSuccess) e = launch_ragged(s.d_data, s.d_offsets, s.d_lengths, count, s.d_crcs, s.stream, s.fault.dev);
    if (e == hipSuccess)
      e = hipMemcpyAsync(s.h_crcs, s.d_crcs, count * sizeof(uint32_t), hipMemcpyDeviceToHost, s.stream);
  }
  if (e == hipSuccess) e = hipEventRecord(s.done, s.stream);
  if (e != hipSuccess) {
    (void)hipStreamSynchronize(s.stream);  // nothing queued may outlive the failed submit
    std::lock_guard<std::mutex> lk(r->lock);
    s.busy = false;
    return fail_hip(e);
  }
  return ENET_CRC_OK;
}

int enet_crc_ring_wait(enet_crc_ring* r, uint32_t slot) {
  if (!r || slot >= r->slots.size()) return ENET_CRC_E_INVALID;
  RingSlot& s = r->slots[slot];
  {
    std::lock_guard<std::mutex> lk(r->lock);
    // Already waited for (or never submitted): the word still holds the last submit's outcome
    // (cleared only by the next submit), so a second wait reports what the first did.
    if (!s.busy) return faulted(s.fault) ? ENET_CRC_E_DEVICE : ENET_CRC_OK;
  }
  DeviceGuard g(r->device);
  const hipError_t e = hipEventSynchronize(s.done);
  {
    std::lock_guard<std::mutex> lk(r->lock);
    s.busy = false;
  }
  if (e != hipSuccess) return fail_hip(e);
  return faulted(s.fault) ? ENET_CRC_E_DEVICE : ENET_CRC_OK;
}

}  // extern "C"

// ---------------------------------------------------------------------------------
// Range coder (include/enet_range_amd.h; kernels in range_coder.hip).

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
  const hipStream_t stream = static_cast<hipStream_t>(hip_stream);
  DeviceGuard g(stream_device(stream));
  hipError_t e = launch_range(decompress, static_cast<const uint8_t*>(d_in), d_in_offsets, d_in_lengths, count,
                              static_cast<uint8_t*>(d_out), d_out_offsets, d_out_limits, d_sizes, d_scratch, workers,
                              stream);
  return e == hipSuccess ? ENET_CRC_OK : fail_hip(e);
}

namespace {

// Host-memory range-coder batch on lane 0 of `ctx` (caller holds the context lock).
// Packet p's input is in_len[p] bytes at h_in + in_off[p] (h_in == NULL: the bytes are
// already in R.in.h at in_off[p]); its output goes to h_out + out_off[p], at most
// out_lim[p] bytes; sizes[p] = the coder's return value.  Only the first sizes[p]
// bytes of each output window are written.
int range_host(enet_crc_ctx* ctx, bool decompress, const uint8_t* h_in, const uint64_t* in_off,
               const uint32_t* in_len, uint64_t count, uint8_t* h_out, const uint64_t* out_off,
               const uint32_t* out_lim, uint32_t* sizes) {
  if (count == 0) return ENET_CRC_OK;
  Lane& L = ctx->lanes[0];
  RangeStage& R = L.range;
  DeviceGuard g(L.device);
  quiesce(L);
  const hipStream_t st = L.slot[0].stream;
  uint64_t ilo = UINT64_MAX, ihi = 0, olo = UINT64_MAX, ohi = 0;
  for (uint64_t p = 0; p < count; ++p) {
    ilo = std::min(ilo, in_off[p]);
    ihi = std::max(ihi, in_off[p] + in_len[p]);
    olo = std::min(olo, out_off[p]);
    ohi = std::max(ohi, out_off[p] + out_lim[p]);
  }
  if (h_in == nullptr) ilo = 0;  // staged at its own offsets
  const size_t ispan = (size_t)(ihi - ilo), ospan = (size_t)(ohi - olo);
  if (h_in) ENET_TRY(R.in.grow(std::max<size_t>(ispan, 1), 16));
  ENET_TRY(R.out.grow(std::max<size_t>(ospan, 1), 16));
  ENET_TRY(R.in_off.grow(count));
  ENET_TRY(R.out_off.grow(count));
  ENET_TRY(R.in_len.grow(count));
  ENET_TRY(R.out_lim.grow(count));
  ENET_TRY(R.sizes.grow(count));
  const uint64_t workers = std::min<uint64_t>(count, kRangeHostWorkers);
  if (workers > R.workers) {
    if (R.d_scratch) (void)hipFree(R.d_scratch);
    R.d_scratch = nullptr;
    R.workers = 0;
    ENET_HIP_TRY(hipMalloc(&R.d_scratch, workers * kRangeArenaBytes));
    R.workers = workers;
  }
  if (h_in) memcpy(R.in.h, h_in + ilo, ispan);
  for (uint64_t p = 0; p < count; ++p) {
    R.in_off.h[p] = in_off[p] - ilo;
    R.in_len.h[p] = in_len[p];
    R.out_off.h[p] = out_off[p] - olo;
    R.out_lim.h[p] = out_lim[p];
  }
  L.slot[0].busy = true;  // quiesce() waits for this stream on an error exit
  ENET_HIP_TRY(hipMemcpyAsync(R.in.d, R.in.h, std::max<size_t>(ispan, 1), hipMemcpyHostToDevice, st));
  ENET_HIP_TRY(hipMemcpyAsync(R.in_off.d, R.in_off.h, count * 8, hipMemcpyHostToDevice, st));
  ENET_HIP_TRY(hipMemcpyAsync(R.in_len.d, R.in_len.h, count * 4, hipMemcpyHostToDevice, st));
  ENET_HIP_TRY(hipMemcpyAsync(R.out_off.d, R.out_off.h, count * 8, hipMemcpyHostToDevice, st));
  ENET_HIP_TRY(hipMemcpyAsync(R.out_lim.d, R.out_lim.h, count * 4, hipMemcpyHostToDevice, st));
  ENET_HIP_TRY(launch_range(decompress, R.in.d, R.in_off.d, R.in_len.d, count, R.out.d, R.out_off.d, R.out_lim.d,
                            R.sizes.d, R.d_scratch, R.workers, st));
  ENET_HIP_TRY(hipMemcpyAsync(R.sizes.h, R.sizes.d, count * 4, hipMemcpyDeviceToHost, st));
  if (ospan) ENET_HIP_TRY(hipMemcpyAsync(R.out.h, R.out.d, ospan, hipMemcpyDeviceToHost, st));
  ENET_HIP_TRY(hipStreamSynchronize(st));
  L.slot[0].busy = false;
  for (uint64_t p = 0; p < count; ++p) {
    const uint32_t n = std::min(R.sizes.h[p], out_lim[p]);
    sizes[p] = R.sizes.h[p];
    if (n) memcpy(h_out + out_off[p], R.out.h + R.out_off.h[p], n);
  }
  return ENET_CRC_OK;
}

}  // namespace

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

int enet_range_compress_iov(enet_crc_ctx* ctx, const enet_crc_iov* bufs, size_t nbufs, size_t in_limit,
                            uint8_t* out, size_t out_limit, size_t* out_size) {
  if (!ctx || !out_size || (nbufs > 0 && !bufs) || (out_limit > 0 && !out)) return ENET_CRC_E_INVALID;
  *out_size = 0;
  if (out_limit > 0xFFFFFFFFull) out_limit = 0xFFFFFFFFull;  // the window is u32-sized
  // compress.rs:79: no slices or a zero in_limit codes nothing.
  if (nbufs == 0 || in_limit == 0) return ENET_CRC_OK;
  // The byte sequence compress.rs:103-126 reads: the slices in order, except that an
  // empty slice after the first reads as one 0 byte (NonNull::dangling(), c.rs:79-85).
  size_t total = 0;
  for (size_t i = 0; i < nbufs; ++i) {
    if (bufs[i].len > 0 && !bufs[i].data) return ENET_CRC_E_INVALID;
    total += bufs[i].len ? bufs[i].len : (i > 0 ? 1 : 0);
  }
  if (total > 0xFFFFFFFFull) return ENET_CRC_E_INVALID;
  std::lock_guard<std::mutex> lk(ctx->lock);
  RangeStage& R = ctx->lanes[0].range;
  {
    DeviceGuard g(ctx->lanes[0].device);
    quiesce(ctx->lanes[0]);
    ENET_TRY(R.in.grow(std::max<size_t>(total, 1), 16));
  }
  size_t pos = 0;
  for (size_t i = 0; i < nbufs; ++i) {
    if (bufs[i].len) {
      memcpy(R.in.h + pos, bufs[i].data, bufs[i].len);
      pos += bufs[i].len;
    } else if (i > 0) {
      R.in.h[pos++] = 0;
    }
  }
  const uint64_t off0 = 0;
  const uint32_t len = (uint32_t)total, lim = (uint32_t)out_limit;
  uint32_t size = 0;
  ENET_TRY(range_host(ctx, false, nullptr, &off0, &len, 1, out, &off0, &lim, &size));
  *out_size = size;
  return ENET_CRC_OK;
}

int enet_range_decompress(enet_crc_ctx* ctx, const uint8_t* in, size_t in_len, uint8_t* out, size_t out_limit,
                          size_t* out_size) {
  if (!ctx || !out_size || (in_len > 0 && !in) || (out_limit > 0 && !out)) return ENET_CRC_E_INVALID;
  *out_size = 0;
  if (in_len > 0xFFFFFFFFull) return ENET_CRC_E_INVALID;
  if (out_limit > 0xFFFFFFFFull) out_limit = 0xFFFFFFFFull;
  if (in_len == 0) return ENET_CRC_OK;  // compress.rs:481-483
  std::lock_guard<std::mutex> lk(ctx->lock);
  const uint64_t off0 = 0;
  const uint32_t len = (uint32_t)in_len, lim = (uint32_t)out_limit;
  uint32_t size = 0;
  ENET_TRY(range_host(ctx, true, in, &off0, &len, 1, out, &off0, &lim, &size));
  *out_size = size;
  return ENET_CRC_OK;
}

static int range_ragged_host(enet_crc_ctx* ctx, bool decompress, const void* h_in, const uint64_t* h_in_offsets,
                             const uint32_t* h_in_lengths, uint64_t count, void* h_out,
                             const uint64_t* h_out_offsets, const uint32_t* h_out_limits, uint32_t* h_sizes) {
  if (!ctx) return ENET_CRC_E_INVALID;
  if (count == 0) return ENET_CRC_OK;
  if (!h_in || !h_in_offsets || !h_in_lengths || !h_out || !h_out_offsets || !h_out_limits || !h_sizes)
    return ENET_CRC_E_INVALID;
  std::lock_guard<std::mutex> lk(ctx->lock);
  (void)stop_server_for_batch(ctx);  // a wedged wave only delays one workgroup
  return range_host(ctx, decompress, static_cast<const uint8_t*>(h_in), h_in_offsets, h_in_lengths, count,
                    static_cast<uint8_t*>(h_out), h_out_offsets, h_out_limits, h_sizes);
}

int enet_range_compress_ragged_host(enet_crc_ctx* ctx, const void* h_in, const uint64_t* h_in_offsets,
                                    const uint32_t* h_in_lengths, uint64_t count, void* h_out,
                                    const uint64_t* h_out_offsets, const uint32_t* h_out_limits, uint32_t* h_sizes) {
  return range_ragged_host(ctx, false, h_in, h_in_offsets, h_in_lengths, count, h_out, h_out_offsets, h_out_limits,
                           h_sizes);
}

int enet_range_decompress_ragged_host(enet_crc_ctx* ctx, const void* h_in, const uint64_t* h_in_offsets,
                                      const uint32_t* h_in_lengths, uint64_t count, void* h_out,
                                      const uint64_t* h_out_offsets, const uint32_t* h_out_limits,
                                      uint32_t* h_sizes) {
  return range_ragged_host(ctx, true, h_in, h_in_offsets, h_in_lengths, count, h_out, h_out_offsets, h_out_limits,
                           h_sizes);
}

}  // extern "C"
