// CDNA4 (gfx950) kernels for the ENet per-datagram CRC-32.
//
// Reference: jabuwu/rusty_enet src/crc32.rs:39-47 (one serial Sarwate chain per
// call, one call per datagram from src/c/protocol.rs:1499 / :2287).  Here a batch
// of packets is checksummed in one launch; a GROUP of 8 lanes cooperates on one
// packet and a wavefront holds 8 packets at a time (a "round").
//
// Arithmetic (DESIGN.md §3 has the derivation; tests/cpp/kernel_sim.cpp models it):
//   * The packet is viewed as little-endian 32-bit words on the 4-byte grid that
//     ends at a1 = e & ~3 (crc32_geometry.hpp).  Word d (d = 1 is the last) sits
//     at a1 - 4d; the zero-initialised register after the words is
//         R = XOR_d M32^d (w_d),   M32 = "advance the register over 32 zero bits".
//   * 16-byte chunk c (counted from the end) belongs to lane k = c % 8 at step
//     i = c / 8.  Each lane's 4 word slots are independent Horner streams with
//     step W = 32 words:  h <- M32^32(h) ^ w, through one replicated LDS table.
//     Steps before a packet's top chunk read zeros and leave h = 0.
//   * The top word is masked to the packet's own bytes and the 0xFFFFFFFF initial
//     register is injected by XOR-ing head_k[s & 3] into it.
//   * Round end: in-lane Horner with M32 over the 4 slots, a 3-level DPP tree
//     with fixed shifts M32^4/8/16 across the 8 lanes, one more M32, then Sarwate
//     byte steps for the e & 3 trailing bytes (src/crc32.rs:43) and
//     bswap32(~R) == (!crc).to_be() (src/crc32.rs:46).
//
// Memory pipeline.  Every slot issues exactly one global_load_dwordx4 per lane,
// unconditionally: chunks outside a packet read a zero dummy, so control flow
// between a load and its use is straight-line and hipcc's s_waitcnt counts stay
// exact (no vmcnt(0) drains; see DESIGN.md "waitcnt discipline").
//   crc32_rounds_kernel<NS>: every packet has NS-1..NS steps (uniform batches, or
//     length-bucketed ragged batches).  One loop iteration = one round: consume
//     round r's NS slots while issuing round r+1's NS loads into the same ring
//     registers; descriptors are prefetched two rounds ahead.
//   crc32_stream_kernel<U>: any lengths.  A round is padded to a multiple of U
//     slots and streamed through a U-deep ring; only round boundaries drain.
//
// LDS tables (76.25 KiB, crc32_layout.hpp has the details):
//   [0, 64 KiB)   replicated block: one 256-B row per byte value, holding 8 copies of
//                 the four M32^32 tables (the Horner step) and 8 copies of the four
//                 M32^1 tables (the in-lane combine).  Lane l reads copy l&7 of table
//                 j ^ ((l>>3)&3) in lookup j: the 32 lanes of a ds_read_b32 group hit
//                 32 different banks.  Each address is ONE v_perm_b32.
//   [64 KiB, +)   unreplicated tree operators M32^4/8/16.
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include <atomic>
#include <mutex>
#include <type_traits>
#include <utility>
#include <vector>

#include "crc32_geometry.hpp"
#include "crc32_kernels.hpp"
#include "crc32_layout.hpp"
#include "crc32_ops.hpp"
#include "crc32_slot.hpp"

namespace enet_crc {

__device__ const OpTables g_op_tables = kOpTables;
// Read by every lane whose chunk lies outside its packet; never written.
__device__ __attribute__((aligned(64))) const uint32_t g_zero_chunk[64] = {0};
// The device's per-call server kick word (enet_crc_abi.hip, crc32_mailbox.hpp), or null.
__device__ uint32_t* g_kick_word = nullptr;

hipError_t set_device_kick_word(uint32_t* d_word) {
  return hipMemcpyToSymbol(HIP_SYMBOL(g_kick_word), &d_word, sizeof(d_word));
}

// Failure words (crc32_kernels.hpp: FaultWord): mapped, coherent pinned host memory that a
// ragged jobs launch writes its kFault* bit into, so the host sees it without a copy.  Every
// launch carries the device address of its word (RaggedJobsBatch::fault): a slot of a
// synchronous entry passes its own, the asynchronous entries the device-wide one.
hipError_t alloc_fault_word(FaultWord* w) {
  *w = FaultWord{};
  uint32_t* h = nullptr;
  uint32_t* d = nullptr;
  hipError_t e = hipHostMalloc((void**)&h, 64, hipHostMallocMapped | hipHostMallocCoherent);
  if (e == hipSuccess) {
    memset(h, 0, 64);
    e = hipHostGetDevicePointer((void**)&d, h, 0);
  }
  if (e != hipSuccess) {
    if (h) (void)hipHostFree(h);
    return e;
  }
  w->host = h;
  w->dev = d;
  return hipSuccess;
}

void free_fault_word(FaultWord& w) {
  if (w.host) (void)hipHostFree(const_cast<uint32_t*>(w.host));
  w = FaultWord{};
}

namespace {
constexpr int kMaxFaultDevices = 64;
std::mutex g_fault_lock;
FaultWord g_fault_dev[kMaxFaultDevices];  // each device's word (never freed: 64 B)
}  // namespace

hipError_t device_fault_word(int dev, FaultWord* out) {
  if (dev < 0 || dev >= kMaxFaultDevices) return hipErrorInvalidDevice;
  std::lock_guard<std::mutex> lk(g_fault_lock);
  if (!g_fault_dev[dev].host) {
    int cur = -1;
    hipError_t e = hipGetDevice(&cur);
    if (e != hipSuccess) return e;
    if (cur != dev && (e = hipSetDevice(dev)) != hipSuccess) return e;
    e = alloc_fault_word(&g_fault_dev[dev]);
    if (cur != dev) (void)hipSetDevice(cur);
    if (e != hipSuccess) return e;
  }
  *out = g_fault_dev[dev];
  return hipSuccess;
}

namespace {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
// 16 bytes at a 4-byte-aligned address (global_load_dwordx4; gfx950 runs in
// unaligned-access mode).
struct __attribute__((packed, aligned(4))) U32x4A4 {
  u32x4 v;
};
// Global address space: keeps loads global_load_* (flat_* would also count on
// lgkmcnt and serialise against the LDS table lookups).
typedef __attribute__((address_space(1))) const uint32_t GlobalU32;
typedef __attribute__((address_space(1))) const U32x4A4 GlobalU32x4A4;

constexpr int kBlock = 1024;
constexpr int kWavesPerBlock = kBlock / 64;
constexpr int G = kLanesPerPacket;
constexpr int kStreamDepth = 8;  // ring depth of the streaming kernel
// LDS layout constants, Lookup and make_lookup(): crc32_layout.hpp.

__device__ __forceinline__ uint32_t load_word(uint64_t addr) { return *reinterpret_cast<GlobalU32*>(addr); }
__device__ __forceinline__ u32x4 load_chunk(uint64_t addr) { return reinterpret_cast<GlobalU32x4A4*>(addr)->v; }

// A batch kernel's first thread bumps the device's kick word: a resident per-call server
// wave exits at its next poll and frees its CU for this grid (one workgroup per CU with a
// static share: a workgroup left waiting for that CU would double the launch).  Vector
// load and store with system scope, waited for at once (no scalar-cache writes).
__device__ __forceinline__ void send_servers_home() {
  if (blockIdx.x != 0 || threadIdx.x != 0 || gridDim.x == 1) return;
  uint32_t* const k = g_kick_word;
  if (!k) return;
  uint32_t v;
  asm volatile("global_load_dword %0, %1, off sc0 sc1\n\ts_waitcnt vmcnt(0)" : "=v"(v) : "v"(k) : "memory");
  v += 1u;
  asm volatile("global_store_dword %0, %1, off sc0 sc1\n\ts_waitcnt vmcnt(0)" : : "v"(k), "v"(v) : "memory");
}

__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}

__device__ __forceinline__ uint32_t lds_at(const uint32_t* lds, uint32_t byte_addr) {
  return *reinterpret_cast<const uint32_t*>(reinterpret_cast<const char*>(lds) + byte_addr);
}

// M(h) ^ w through a replicated set (lp = lk.lp: M32^32, lk.lp1: M32^1): 4 v_perm
// (each one byte address) + 4 conflict-free ds_read_b32.
__device__ __forceinline__ uint32_t apply_rep(const uint32_t* lds, uint32_t h, uint32_t w, uint32_t lp,
                                              const Lookup& lk) {
  const uint32_t a0 = lookup_addr(h, lp, lk, 0);
  const uint32_t a1 = lookup_addr(h, lp, lk, 1);
  const uint32_t a2 = lookup_addr(h, lp, lk, 2);
  const uint32_t a3 = lookup_addr(h, lp, lk, 3);
  return xor3(xor3(lds_at(lds, a0), lds_at(lds, a1), lds_at(lds, a2)), lds_at(lds, a3), w);
}

// h' = M32^32(h) ^ w: one Horner step of a word stream.
__device__ __forceinline__ uint32_t horner_main(const uint32_t* lds, uint32_t h, uint32_t w, const Lookup& lk) {
  return apply_rep(lds, h, w, lk.lp, lk);
}

__device__ __forceinline__ uint32_t sarwate_at(const uint32_t* lds, uint32_t idx) {
  return lds[idx * kRowDwords + kSarwateDword];
}

// M32^n(x) through an unreplicated 4x256 table set.
__device__ __forceinline__ uint32_t apply_small(const uint32_t* set, uint32_t x) {
  return xor3(set[x & 0xffu], set[256 + ((x >> 8) & 0xffu)], set[512 + ((x >> 16) & 0xffu)]) ^
         set[768 + (x >> 24)];
}

// Lane l receives lane l+d of its 16-lane DPP row (groups of 8 never straddle a row).
template <int d>
__device__ __forceinline__ uint32_t from_lane_plus(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x100 + d, 0xF, 0xF, true);
}

__device__ __forceinline__ uint32_t head_k(uint32_t v) {
  return v == 0 ? kOpTables.head_k[0]
                : (v == 1 ? kOpTables.head_k[1] : (v == 2 ? kOpTables.head_k[2] : kOpTables.head_k[3]));
}

__device__ __forceinline__ int32_t wave_max_over_groups(int32_t v) {
  int32_t m = __builtin_amdgcn_readlane(v, 0);
#pragma unroll
  for (int g = 1; g < kPacketsPerWave; ++g) m = max(m, __builtin_amdgcn_readlane(v, g * G));
  return m;
}

// The replicated block, written row-linearly: 16-B piece x of the 64-KiB block (row x / 16,
// dwords 4 (x % 16) .. + 3 of the row: 4 copies of one table entry) goes to lane x of the
// store, so consecutive lanes write consecutive 16 B (a lane-per-row order had every lane
// of a ds_write_b128 in the same bank group).  `main` = the Horner operator's level.
// `set0` / `set1`: the operator levels of the block's two sets.
// Every thread issues all its table loads before its first LDS store (TableLoads): as a loop of
// load -> wait -> store, a kernel's start paid one memory latency per iteration, 7 to 10 in a
// row before its first batch load (round 6).
constexpr int kRepPieces = kRepDwords / 4 / kBlock;  // 16-B pieces of the replicated block per thread
static_assert(kRepDwords / 4 % kBlock == 0, "whole pieces per thread");
template <int NT>
struct TableLoads {
  uint32_t rep[kRepPieces];  // one dword per replicated piece
  uint32_t tree[NT];         // unreplicated sets, one dword per 1024
};
__device__ __forceinline__ uint32_t replicated_value(uint32_t x, int set0, int set1) {
  const uint32_t i = x / (kRowDwords / 4), d = 4u * (x % (kRowDwords / 4));  // row (byte value), first dword
  const uint32_t second = d >= kSetM1Bytes / 4 ? 1u : 0u, tab = (d % (kSetM1Bytes / 4)) / kRepCopies;
  return g_op_tables.op[second ? set1 : set0][tab][i];
}
// NT unreplicated sets after the block: set l is M32^(4 * 2^l) (level l + 2).
template <int NT>
__device__ __forceinline__ TableLoads<NT> load_tables(int set0, int set1) {
  TableLoads<NT> t;
#pragma unroll
  for (int r = 0; r < kRepPieces; ++r) t.rep[r] = replicated_value(threadIdx.x + r * kBlock, set0, set1);
#pragma unroll
  for (int r = 0; r < NT; ++r) {
    const uint32_t x = threadIdx.x + r * kBlock, rem = x & 1023u;
    t.tree[r] = g_op_tables.op[(x >> 10) + 2][rem >> 8][rem & 255u];
  }
  return t;
}
template <int NT>
__device__ __forceinline__ void store_tables(uint32_t* lds, uint32_t tree_dword, const TableLoads<NT>& t) {
#pragma unroll
  for (int r = 0; r < kRepPieces; ++r) {
    const uint32_t v = t.rep[r];
    reinterpret_cast<u32x4*>(lds)[threadIdx.x + r * kBlock] = u32x4{v, v, v, v};
  }
#pragma unroll
  for (int r = 0; r < NT; ++r) lds[tree_dword + threadIdx.x + r * kBlock] = t.tree[r];
}
static_assert(kBlock == 1024, "the unreplicated sets are 1024 dwords: one per thread");

__device__ __forceinline__ void fill_lds(uint32_t* lds) {
  store_tables<kTreeLevels>(lds, kTreeDword, load_tables<kTreeLevels>(kMainLevel, 0));
}
// fill_lds's tables by nt >= 768 threads (t = 0 .. nt - 1 here), all loads before the stores.
__device__ __forceinline__ void fill_lds_from(uint32_t* lds, uint32_t t, uint32_t nt) {
  constexpr uint32_t kPieces = kRepDwords / 4, kTree = kTreeLevels * 1024u;
  constexpr int kRepIt = (kPieces + 767) / 768, kTreeIt = (kTree + 767) / 768;
  uint32_t rep[kRepIt], tree[kTreeIt];
#pragma unroll
  for (int r = 0; r < kRepIt; ++r) {
    const uint32_t x = t + r * nt;
    rep[r] = x < kPieces ? replicated_value(x, kMainLevel, 0) : 0u;
  }
#pragma unroll
  for (int r = 0; r < kTreeIt; ++r) {
    const uint32_t x = t + r * nt, rem = x & 1023u;
    tree[r] = x < kTree ? g_op_tables.op[(x >> 10) + 2][rem >> 8][rem & 255u] : 0u;
  }
#pragma unroll
  for (int r = 0; r < kRepIt; ++r) {
    const uint32_t x = t + r * nt, v = rep[r];
    if (x < kPieces) reinterpret_cast<u32x4*>(lds)[x] = u32x4{v, v, v, v};
  }
#pragma unroll
  for (int r = 0; r < kTreeIt; ++r) {
    const uint32_t x = t + r * nt;
    if (x < kTree) lds[kTreeDword + x] = tree[r];
  }
}

template <bool kRagged>
struct Batch {
  uint64_t base;
  const uint64_t* offsets;
  const uint32_t* lengths;
  uint64_t stride;
  uint32_t length;
  uint64_t count;
};

// Packet id processed in position p (past the end: the last packet, read as empty).
template <bool kRagged>
__device__ __forceinline__ uint64_t packet_id(const Batch<kRagged>& b, uint64_t p) {
  if constexpr (kRagged) return p < b.count ? p : b.count - 1;
  return p;
}

// Descriptor of the packet in position p (p >= count reads as an empty packet).
template <bool kRagged>
__device__ __forceinline__ void load_desc(const Batch<kRagged>& b, uint64_t p, uint64_t& off, uint32_t& len) {
  if constexpr (kRagged) {
    const uint64_t q = packet_id(b, p);
    off = b.offsets[q];
    len = p < b.count ? b.lengths[q] : 0;
  } else {
    off = (p < b.count ? p : 0) * b.stride;
    len = p < b.count ? b.length : 0;
  }
}

// Round-constant slot metadata for one lane (bit layout private to this file).
constexpr uint32_t kMetaHeadMask = 0x7;       // c != 0: top word at word index 4 - c of the top chunk
constexpr uint32_t kMetaVShift = 3;           // 2 bits: sa - top
constexpr uint32_t kMetaEmpty = 1u << 5;      // packet has no grid word: register = init
constexpr uint32_t kMetaNTailShift = 6;       // 2 bits: trailing bytes (0..3)
constexpr uint32_t kMetaTShiftShift = 8;      // 2 bits: first trailing byte's position in its word
constexpr uint32_t kMetaStore = 1u << 10;     // packet index < count
constexpr uint32_t kMetaFallback = 1u << 11;  // top chunk begins before the caller's buffer
constexpr uint32_t kMetaDirect = 1u << 12;    // ragged rounds: the top chunk is read directly (inside, no fallback)
constexpr uint32_t kMetaLineRShift = 8;       // line rounds: 2 bits, r = (E16 - a1) / 4 words (ragged rounds
                                              // never use kMetaTShiftShift's field)
constexpr uint32_t kMetaSkipShift = 15;       // line rounds: 4 bits, words not multiplied in at the last slot
constexpr uint32_t kHeadZero = 5;             // line rounds: head code of a chunk wholly before the first word

__device__ __forceinline__ uint32_t round_meta(const PacketGeo& g, uint32_t k, uint64_t base4, bool store,
                                               uint64_t& tail_addr, uint64_t dummy) {
  uint32_t head = 0, fb = 0;
  if (g.nsteps > 0) {
    const int32_t itop = g.nsteps - 1;
    const int64_t rel0 = chunk_offset(g, k, itop, g.top);
    head = (rel0 > -16 && rel0 <= 0) ? (uint32_t)(rel0 / 4 + 4) : 0u;
    fb = chunk_kind(g, k, itop, base4) == kChunkFallback ? kMetaFallback : 0u;
  }
  const uint64_t ts = g.a1 > g.sa ? g.a1 : g.sa;
  const uint32_t ntail = (uint32_t)(g.ea - ts);
  tail_addr = ntail ? g.a1 : dummy;
  return head | ((uint32_t)(g.sa - g.top) << kMetaVShift) | (g.nsteps == 0 ? kMetaEmpty : 0u) |
         (ntail << kMetaNTailShift) | ((uint32_t)(ts - g.a1) << kMetaTShiftShift) | (store ? kMetaStore : 0u) | fb;
}

// Top chunk words: keep only the packet's own bytes and inject the initial register.
__device__ __forceinline__ void mask_top(uint32_t meta, uint32_t& w0, uint32_t& w1, uint32_t& w2, uint32_t& w3) {
  const uint32_t head = meta & kMetaHeadMask;
  const uint32_t v = (meta >> kMetaVShift) & 3u;
  const uint32_t keep = 0xFFFFFFFFu << (8u * v), kk = head_k(v);
  const int32_t j0 = 4 - (int32_t)head;  // word index of the top word
  w0 = j0 > 0 ? 0 : (j0 == 0 ? (w0 & keep) ^ kk : w0);
  w1 = j0 > 1 ? 0 : (j0 == 1 ? (w1 & keep) ^ kk : w1);
  w2 = j0 > 2 ? 0 : (j0 == 2 ? (w2 & keep) ^ kk : w2);
  w3 = j0 == 3 ? (w3 & keep) ^ kk : w3;
}

// Fallback for a top chunk that begins before the caller's buffer: read only the
// words at or after the chunk's top word (rare: packets within 12 bytes of base).
// One asm statement issues the loads AND waits for them, so hipcc sees a plain
// definition of w0..w3: no pending load on this rare path can leak into the waitcnt
// bookkeeping of the ring registers (which would turn every slot's wait into a
// vmcnt(0) drain).
__device__ __forceinline__ void load_top_words(uint64_t chunk_addr, uint32_t meta, uint64_t dummy, uint32_t& w0,
                                               uint32_t& w1, uint32_t& w2, uint32_t& w3) {
  const int32_t j0 = 4 - (int32_t)(meta & kMetaHeadMask);
  const uint64_t a0 = j0 <= 0 ? chunk_addr : dummy;
  const uint64_t a1 = j0 <= 1 ? chunk_addr + 4 : dummy;
  const uint64_t a2 = j0 <= 2 ? chunk_addr + 8 : dummy;
  const uint64_t a3 = chunk_addr + 12;
  asm volatile(
      "global_load_dword %0, %4, off\n\t"
      "global_load_dword %1, %5, off\n\t"
      "global_load_dword %2, %6, off\n\t"
      "global_load_dword %3, %7, off\n\t"
      "s_waitcnt vmcnt(0)"
      : "=&v"(w0), "=&v"(w1), "=&v"(w2), "=&v"(w3)
      : "v"(a0), "v"(a1), "v"(a2), "v"(a3)
      : "memory");
}

// Combine the 4 word streams of each of the group's 8 lanes into y, the packet's
// register before the shift of its last word (register = M32 y).  Valid on lane k == 0.
__device__ __forceinline__ uint32_t combine_tree(const uint32_t* lds, uint32_t h0, uint32_t h1, uint32_t h2,
                                                uint32_t h3, const Lookup& lk) {
  // In-lane Horner over the 4 word slots with M32^1 (replicated: conflict-free).
  uint32_t y = apply_rep(lds, h0, h1, lk.lp1, lk);
  y = apply_rep(lds, y, h2, lk.lp1, lk);
  y = apply_rep(lds, y, h3, lk.lp1, lk);
  // Tree levels: only the lanes whose value moves down look it up (the others are
  // masked off, which also keeps them out of the unreplicated tables' bank conflicts).
  const uint32_t k = threadIdx.x & (G - 1);
  uint32_t t = 0;
  if (k & 1u) t = apply_small(lds + kTreeDword, y);
  y ^= from_lane_plus<1>(t);
  if ((k & 3u) == 2u) t = apply_small(lds + kTreeDword + 1024, y);
  y ^= from_lane_plus<2>(t);
  if (k == 4u) t = apply_small(lds + kTreeDword + 2048, y);
  y ^= from_lane_plus<4>(t);
  return y;
}

// combine_tree's three tree levels for a kernel whose tables start at LDS address 0 (the
// unreplicated tree sets at kTreeDword, byte 0x10000).  Each lookup address is ONE
// v_lshlrev_b32_sdwa: byte j of y, times 4, written into the low half of `a`, whose high half
// always holds 1 (dst_unused:UNUSED_PRESERVE), plus the set and table in the ds_read offset
// (hipcc: v_bfe + v_lshl_or with the table base in a VGPR per table, 2 VALU per lookup).  The
// levels' lane masks are set with scalar moves instead of hipcc's per-level saveexec of a
// hoisted (and spilled to VGPR lanes) compare.  EXEC is all ones on entry (the round loop).
// Lanes whose value does not move keep stale t; only lane k == 0's y is meaningful at the end.
// Hazards (not inserted for inline asm): a VALU write then a DPP read of that VGPR needs 2
// wait states (s_nop 1).
#define ENET_TREE_LEVEL(MASK, OFF0, OFF1, OFF2, OFF3, SHL)                                                      \
  "s_mov_b32 exec_lo, " MASK "\n\ts_mov_b32 exec_hi, " MASK "\n\t"                                             \
  "v_lshlrev_b32_sdwa %[a], 2, %[y] dst_sel:WORD_0 dst_unused:UNUSED_PRESERVE src0_sel:DWORD src1_sel:BYTE_0\n\t" \
  "ds_read_b32 %[t0], %[a] offset:" OFF0 "\n\t"                                                                 \
  "v_lshlrev_b32_sdwa %[a], 2, %[y] dst_sel:WORD_0 dst_unused:UNUSED_PRESERVE src0_sel:DWORD src1_sel:BYTE_1\n\t" \
  "ds_read_b32 %[t1], %[a] offset:" OFF1 "\n\t"                                                                 \
  "v_lshlrev_b32_sdwa %[a], 2, %[y] dst_sel:WORD_0 dst_unused:UNUSED_PRESERVE src0_sel:DWORD src1_sel:BYTE_2\n\t" \
  "ds_read_b32 %[t2], %[a] offset:" OFF2 "\n\t"                                                                 \
  "v_lshlrev_b32_sdwa %[a], 2, %[y] dst_sel:WORD_0 dst_unused:UNUSED_PRESERVE src0_sel:DWORD src1_sel:BYTE_3\n\t" \
  "ds_read_b32 %[t3], %[a] offset:" OFF3 "\n\t"                                                                 \
  "s_waitcnt lgkmcnt(0)\n\t"                                                                                    \
  "v_bitop3_b32 %[t0], %[t0], %[t1], %[t2] bitop3:0x96\n\t"                                                     \
  "v_xor_b32 %[t0], %[t0], %[t3]\n\t"                                                                           \
  "s_mov_b64 exec, %[sv]\n\t"                                                                                   \
  "s_nop 1\n\t"                                                                                                 \
  "v_xor_b32_dpp %[y], %[t0], %[y] row_shl:" SHL " row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
__device__ __forceinline__ uint32_t tree_levels_asm(uint32_t y, uint32_t& a) {
  static_assert(kTreeDword * 4u == 0x10000u && kTreeLevels == 3, "the asm's addresses");
  uint32_t t0, t1, t2, t3;
  uint64_t sv;
  asm volatile("s_mov_b64 %[sv], exec\n\t"
               // M32^4: lanes k = 1, 3, 5, 7 of each group of 8, into k - 1
               ENET_TREE_LEVEL("0xAAAAAAAA", "0", "1024", "2048", "3072", "1")
               // M32^8: lanes k = 2, 6, into k - 2
               ENET_TREE_LEVEL("0x44444444", "4096", "5120", "6144", "7168", "2")
               // M32^16: lane k = 4, into k = 0
               ENET_TREE_LEVEL("0x10101010", "8192", "9216", "10240", "11264", "4")
               : [y] "+v"(y), [a] "+v"(a), [t0] "=&v"(t0), [t1] "=&v"(t1), [t2] "=&v"(t2), [t3] "=&v"(t3),
                 [sv] "=&s"(sv)
               :
               : "memory");
  return y;
}
#undef ENET_TREE_LEVEL

// combine_tree for the register-ring kernel's layout (kRegsLdsDwords): the first two tree
// levels through the replicated tree block (conflict-free), the third unreplicated.
__device__ __forceinline__ uint32_t combine_tree_rep(const uint32_t* lds, uint32_t h0, uint32_t h1, uint32_t h2,
                                                    uint32_t h3, const Lookup& lk) {
  uint32_t y = apply_rep(lds, h0, h1, lk.lp1, lk);
  y = apply_rep(lds, y, h2, lk.lp1, lk);
  y = apply_rep(lds, y, h3, lk.lp1, lk);
  const uint32_t k = threadIdx.x & (G - 1);
  uint32_t t = 0;
  if (k & 1u) t = apply_rep(lds + kTreeRepDword, y, 0u, lk.lp, lk);  // M32^4
  y ^= from_lane_plus<1>(t);
  if ((k & 3u) == 2u) t = apply_rep(lds + kTreeRepDword, y, 0u, lk.lp1, lk);  // M32^8
  y ^= from_lane_plus<2>(t);
  if (k == 4u) t = apply_small(lds + kTree16Dword, y);  // M32^16
  y ^= from_lane_plus<4>(t);
  return y;
}

// The register kernels' tables: the main block, the replicated tree block (M32^4 and M32^8)
// and the unreplicated M32^16 set; every load issued before any store (TableLoads).  Split in
// two so that a kernel can issue its first batch loads between them.
struct RegsTableLoads {
  TableLoads<0> main, tree;
  uint32_t t16;
};
__device__ __forceinline__ RegsTableLoads load_regs_tables() {
  RegsTableLoads t;
  t.main = load_tables<0>(kMainLevel, 0);
  t.tree = load_tables<0>(2, 3);
  const uint32_t x = threadIdx.x;
  t.t16 = g_op_tables.op[4][x >> 8][x & 255u];
  return t;
}
__device__ __forceinline__ void store_regs_tables(uint32_t* lds, const RegsTableLoads& t) {
  store_tables<0>(lds, 0, t.main);
  store_tables<0>(lds + kTreeRepDword, 0, t.tree);
  lds[kTree16Dword + threadIdx.x] = t.t16;
}
__device__ __forceinline__ void fill_lds_regs(uint32_t* lds) { store_regs_tables(lds, load_regs_tables()); }

// The packet's register (before trailing bytes), valid on lane k == 0 of the group.
__device__ __forceinline__ uint32_t combine_streams(const uint32_t* lds, uint32_t h0, uint32_t h1, uint32_t h2,
                                                   uint32_t h3, const Lookup& lk) {
  const uint32_t y = combine_tree(lds, h0, h1, h2, h3, lk);
  return apply_rep(lds, y, 0u, lk.lp1, lk);  // every lane (conflict-free); lane k == 0 holds the register
}

// The register of a packet the DMA kernels ran z = 0..3 zero bytes past its end (to the
// next 4-byte boundary), from the tree value y: M8^-z M32 y = M8^m y with m = 4 - z, so
// the last word's shift simply stops z bytes short.  Byte j of y reaches position 0
// only if j < m, so
//     M8^m(y) = M32(y << 8z) ^ (y >> (32 - 8z))      (second term 0 for z = 0):
// the bytes that never reach the bottom leave unchanged, the others go through the
// ordinary M32^1 lookups (one apply_rep: the lane's own conflict-free copies and
// selectors, so it runs on every lane without masking; lane k == 0's value is used).
__device__ __forceinline__ uint32_t finish_word(const uint32_t* lds, uint32_t y, uint32_t z, const Lookup& lk) {
  const uint32_t lo = y << (8u * z);
  const uint32_t hi = z ? y >> (32u - 8u * z) : 0u;
  return apply_rep(lds, lo, hi, lk.lp1, lk);
}

// Sarwate byte steps (src/crc32.rs:43) over `ntail` bytes of `word` from byte `tsh`.
__device__ __forceinline__ uint32_t tail_steps(const uint32_t* lds, uint32_t reg, uint32_t word, uint32_t ntail,
                                               uint32_t tsh) {
#pragma unroll
  for (uint32_t t = 0; t < 3; ++t) {
    if (t < ntail) reg = (reg >> 8) ^ sarwate_at(lds, (reg ^ (word >> (8u * (tsh + t)))) & 0xffu);
  }
  return reg;
}

// Round end: combine the 4x8 streams, trailing bytes, store (lane 0 of the group).
__device__ __forceinline__ void finish_round(const uint32_t* lds, uint32_t h0, uint32_t h1, uint32_t h2, uint32_t h3,
                                             uint32_t meta, uint32_t tail_word, uint32_t k, const Lookup& lk,
                                             uint32_t* dst) {
  uint32_t reg = combine_streams(lds, h0, h1, h2, h3, lk);
  if (meta & kMetaEmpty) reg = kInitRegister;
  reg = tail_steps(lds, reg, tail_word, (meta >> kMetaNTailShift) & 3u, (meta >> kMetaTShiftShift) & 3u);
  if (k == 0 && (meta & kMetaStore)) *dst = __builtin_bswap32(~reg);
}

// Ring loads must issue in slot order: hipcc's scheduler otherwise reorders the
// independent loads of a loop body (it reversed them), the ring order breaks, and the
// loop-header merge of the waitcnt scoreboard degrades every slot's wait to vmcnt(1).
__device__ __forceinline__ void issue_order_fence() { __builtin_amdgcn_sched_barrier(0); }

struct LaneConsts {
  uint32_t k, grp;
  Lookup lk;
  uint64_t base4, dummy;
};

__device__ __forceinline__ LaneConsts lane_consts(uint64_t base) {
  LaneConsts c;
  const uint32_t lane = threadIdx.x & 63u;
  c.k = lane & (G - 1);
  c.grp = lane / G;
  c.lk = make_lookup(lane);
  c.base4 = base & ~(uint64_t)3;
  c.dummy = (uint64_t)(uintptr_t)g_zero_chunk;
  return c;
}

// ---------------------------------------------------------------------------------
// Round kernel: every packet of the launch has at most NS steps.
// ---------------------------------------------------------------------------------
template <int NS>
struct RoundPlan {
  uint64_t base;       // this lane's chunk address at slot 0 (step NS-1)
  uint32_t vmask;      // bit s: slot s reads real data
  uint32_t meta;       // round_meta()
  int32_t top_slot;    // slot of the group's top step (NS: none)
  uint64_t tail_addr;  // word holding the trailing bytes, or the dummy
};

template <int NS>
__device__ __forceinline__ RoundPlan<NS> plan_round(const PacketGeo& g, const LaneConsts& c, bool store) {
  RoundPlan<NS> pl;
  pl.base = g.a1 - 16u * (uint64_t)(c.k + 1u) - (uint64_t)kBytesPerStep * (NS - 1);
  pl.meta = round_meta(g, c.k, c.base4, store, pl.tail_addr, c.dummy);
  pl.top_slot = NS - g.nsteps;  // g.nsteps <= NS by the launch contract
  uint32_t vm = 0;
  if (g.nsteps > 0) {
    const int kind = chunk_kind(g, c.k, g.nsteps - 1, c.base4);
    vm = ((1u << NS) - 1u) & ~((2u << pl.top_slot) - 1u);  // slots after the top one
    if (kind == kChunkDirect) vm |= 1u << pl.top_slot;
  }
  pl.vmask = vm;
  return pl;
}

template <int NS>
__device__ __forceinline__ uint64_t slot_addr(const RoundPlan<NS>& pl, int s, uint64_t dummy) {
  return (pl.vmask >> s) & 1u ? pl.base + (uint64_t)kBytesPerStep * s : dummy;
}

template <int NS, bool kRagged>
__global__ __launch_bounds__(kBlock) void crc32_rounds_kernel(Batch<kRagged> b, uint32_t* __restrict__ out) {
  send_servers_home();
  __shared__ __attribute__((aligned(16))) uint32_t lds[kLdsDwords];
  fill_lds(lds);
  __syncthreads();
  const LaneConsts c = lane_consts(b.base);

  const uint32_t wave = __builtin_amdgcn_readfirstlane(blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6));
  const uint64_t first = (uint64_t)wave * kPacketsPerWave;
  const uint64_t P = (uint64_t)gridDim.x * kWavesPerBlock * kPacketsPerWave;
  if (first >= b.count) return;
  const uint64_t nrounds = (b.count - first + P - 1) / P;

  uint64_t d_off;
  uint32_t d_len;
  load_desc(b, first + c.grp, d_off, d_len);
  RoundPlan<NS> cur = plan_round<NS>(make_geo(b.base + d_off, d_len), c, first + c.grp < b.count);
  load_desc(b, first + P + c.grp, d_off, d_len);  // round 1, consumed one iteration later

  u32x4 q[NS];
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    q[s] = load_chunk(slot_addr(cur, s, c.dummy));
    issue_order_fence();
  }
  uint32_t tw_cur = load_word(cur.tail_addr);

  for (uint64_t r = 0; r < nrounds; ++r) {
    // Producer side: plan round r+1 and prefetch round r+2's descriptor.
    const uint64_t pn = first + (r + 1) * P + c.grp;
    const RoundPlan<NS> nxt = plan_round<NS>(make_geo(b.base + d_off, d_len), c, pn < b.count);
    load_desc(b, pn + P, d_off, d_len);

    uint32_t h0 = 0, h1 = 0, h2 = 0, h3 = 0;
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      uint32_t w0 = q[s].x, w1 = q[s].y, w2 = q[s].z, w3 = q[s].w;
      const bool top = s == cur.top_slot;
      if (__builtin_amdgcn_ballot_w64(top && (cur.meta & kMetaHeadMask))) {
        if (__builtin_amdgcn_ballot_w64(top && (cur.meta & kMetaFallback))) {
          if (top && (cur.meta & kMetaFallback))
            load_top_words(cur.base + (uint64_t)kBytesPerStep * s, cur.meta, c.dummy, w0, w1, w2, w3);
        }
        if (top && (cur.meta & kMetaHeadMask)) mask_top(cur.meta, w0, w1, w2, w3);
      }
      if (s == 0) {  // M32^32(0) = 0: the first step needs no lookups
        h0 = w0; h1 = w1; h2 = w2; h3 = w3;
      } else {
        h0 = horner_main(lds, h0, w0, c.lk);
        h1 = horner_main(lds, h1, w1, c.lk);
        h2 = horner_main(lds, h2, w2, c.lk);
        h3 = horner_main(lds, h3, w3, c.lk);
      }
      q[s] = load_chunk(slot_addr(nxt, s, c.dummy));
      issue_order_fence();
    }
    const uint32_t tw_next = load_word(nxt.tail_addr);
    finish_round(lds, h0, h1, h2, h3, cur.meta, tw_cur, c.k, c.lk, out + (first + r * P + c.grp));
    cur = nxt;
    tw_cur = tw_next;
  }
}

// ---------------------------------------------------------------------------------
// Streaming kernel: any packet lengths.  Each round (8 packets of a wave) is padded
// to T = ceil(max nsteps / U) * U slots and streamed through a U-deep ring.
// ---------------------------------------------------------------------------------
// The rounds of one wave (`lds` filled by fill_lds).
template <int U, bool kRagged>
__device__ __forceinline__ void stream_rounds(const uint32_t* lds, const Batch<kRagged>& b, uint32_t* __restrict__ out) {
  const LaneConsts c = lane_consts(b.base);

  const uint32_t wave = __builtin_amdgcn_readfirstlane(blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6));
  const uint64_t first = (uint64_t)wave * kPacketsPerWave;
  const uint64_t P = (uint64_t)gridDim.x * kWavesPerBlock * kPacketsPerWave;
  if (first >= b.count) return;
  const uint64_t nrounds = (b.count - first + P - 1) / P;

  for (uint64_t r = 0; r < nrounds; ++r) {
    const uint64_t p = first + r * P + c.grp;
    uint64_t off;
    uint32_t len;
    load_desc(b, p, off, len);
    const PacketGeo g = make_geo(b.base + off, len);
    uint64_t tail_addr;
    const uint32_t meta = round_meta(g, c.k, c.base4, p < b.count, tail_addr, c.dummy);
    const uint32_t tail_word = load_word(tail_addr);
    const int32_t iters = (wave_max_over_groups(g.nsteps) + U - 1) / U;
    const int32_t nslots = iters * U;
    // Slot j reads step i = nslots-1-j; this lane's chunk at step i is
    // a1 - 16(k+1) - 128 i: real data for i < nsteps-1 (and i = nsteps-1 when direct).
    const uint64_t base = g.a1 - 16u * (uint64_t)(c.k + 1u) - (uint64_t)kBytesPerStep * (uint64_t)(nslots - 1);
    const int32_t top_slot = nslots - g.nsteps;  // == nslots when the packet is empty
    const bool top_direct = g.nsteps > 0 && chunk_kind(g, c.k, g.nsteps - 1, c.base4) == kChunkDirect;
    auto addr_of = [&](int32_t j) -> uint64_t {
      const bool real = j > top_slot || (j == top_slot && top_direct);
      return real ? base + (uint64_t)kBytesPerStep * (uint64_t)j : c.dummy;
    };
    u32x4 q[U];
#pragma unroll
    for (int s = 0; s < U; ++s) {
      q[s] = load_chunk(addr_of(s));
      issue_order_fence();
    }
    uint32_t h0 = 0, h1 = 0, h2 = 0, h3 = 0;
    for (int32_t it = 0; it < iters; ++it) {
#pragma unroll
      for (int s = 0; s < U; ++s) {
        const int32_t j = it * U + s;
        uint32_t w0 = q[s].x, w1 = q[s].y, w2 = q[s].z, w3 = q[s].w;
        const bool top = j == top_slot;
        if (__builtin_amdgcn_ballot_w64(top && (meta & kMetaHeadMask))) {
          if (__builtin_amdgcn_ballot_w64(top && (meta & kMetaFallback))) {
            if (top && (meta & kMetaFallback))
              load_top_words(base + (uint64_t)kBytesPerStep * (uint64_t)j, meta, c.dummy, w0, w1, w2, w3);
          }
          if (top && (meta & kMetaHeadMask)) mask_top(meta, w0, w1, w2, w3);
        }
        h0 = horner_main(lds, h0, w0, c.lk);
        h1 = horner_main(lds, h1, w1, c.lk);
        h2 = horner_main(lds, h2, w2, c.lk);
        h3 = horner_main(lds, h3, w3, c.lk);
        q[s] = load_chunk(j + U < nslots ? addr_of(j + U) : c.dummy);
        issue_order_fence();
      }
    }
    finish_round(lds, h0, h1, h2, h3, meta, tail_word, c.k, c.lk, out + packet_id(b, p));
  }
}

template <int U, bool kRagged>
__global__ __launch_bounds__(kBlock) void crc32_stream_kernel(Batch<kRagged> b, uint32_t* __restrict__ out) {
  send_servers_home();
  __shared__ __attribute__((aligned(16))) uint32_t lds[kLdsDwords];
  fill_lds(lds);
  __syncthreads();
  stream_rounds<U, kRagged>(lds, b, out);
}

constexpr int kStepClasses = 16;  // ragged sort key: class = min(nsteps, 15)


// A packet's record (ragged_record; written by the job build of crc32_ragged_jobs_kernel
// into LDS, 12 B per packet): its geometry precomputed so that the round derives every
// lane's plan with 32-bit arithmetic.
//   ax   (u64): a1 | v << 48 | z << 50 | near << 52 | 1 << 53 | local id << 54
//               a1 = end of the packet run to the next 4-byte boundary (z = 0..3 bytes
//               past the end), v = sa & 3, near = top within 16 B of the caller's base
//               (only then can a top chunk need the fallback), bit 53 = a packet is here
//   info (u32): nsteps | (pad / 4) << 26, pad = 128 nsteps - 4 nwords
// (GPU virtual addresses are below 2^48.)
constexpr uint64_t kRecAddrMask = (1ull << 48) - 1;
constexpr int kRecVShift = 48, kRecZShift = 50, kRecNearBit = 52, kRecValidBit = 53;
constexpr uint32_t kRecStepsMask = (1u << 26) - 1;
constexpr int kRecPadShift = 26;
constexpr int kJobLidShift = 54;  // job build: the packet's local id (0..255) in ax bits 54..61
struct RaggedRecord {
  uint64_t ax;
  uint32_t info;
  uint32_t nsteps;
};

__device__ __forceinline__ RaggedRecord ragged_record(uint64_t sa, uint32_t len, uint64_t base4) {
  // make_geo(sa, len + z) in 32-bit words where the values allow it: v + len + z is a multiple
  // of 4 (0 for an empty packet), so nwords = (v + len + z) / 4 without a 64-bit subtraction.
  const uint32_t v = (uint32_t)sa & 3u;
  const uint32_t z = len ? (4u - (((uint32_t)sa + len) & 3u)) & 3u : 0u;
  const uint32_t nwords = (len >> 2) + (((len & 3u) + v + z) >> 2);
  const uint32_t nsteps = (((nwords + 3u) >> 2) + (uint32_t)kLanesPerPacket - 1u) / (uint32_t)kLanesPerPacket;
  const uint32_t pad = 128u * nsteps - 4u * nwords;  // 0..124
  const uint64_t top = sa & ~(uint64_t)3, a1 = top + 4ull * nwords;
  const uint64_t near = top - base4 < 16 ? 1ull : 0ull;
  RaggedRecord r;
  r.ax = a1 | ((uint64_t)v << kRecVShift) | ((uint64_t)z << kRecZShift) | (near << kRecNearBit) |
         (1ull << kRecValidBit);
  r.info = nsteps | ((pad >> 2) << kRecPadShift);
  r.nsteps = nsteps;
  return r;
}

// Inclusive prefix sum over the 64 lanes in DPP (no LDS round trips): shifts of 1, 2, 4
// and 8 inside each 16-lane row, then row 0's and row 1's last lanes broadcast into the
// rows above (row_bcast:15 into rows 1 and 3, row_bcast:31 into rows 2 and 3).
__device__ __forceinline__ uint32_t wave_inclusive_add(uint32_t x) {
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xf, 0xf, true);  // row_shr:1
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xf, 0xf, true);  // row_shr:2
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xf, 0xf, true);  // row_shr:4
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xf, 0xf, true);  // row_shr:8
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xa, 0xf, false);  // row_bcast:15
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xc, 0xf, false);  // row_bcast:31
  return x;
}

// Uniform batches: base and stride multiples of 4, so every packet has the same
// geometry relative to its own start.
struct UniformBatch {
  uint64_t base;
  uint64_t stride;
  uint32_t length;
  uint64_t count;
  // crc32_uniform_regs_kernel only: packets p >= skip_at are packets p + skip of the batch
  // (address and output), so one launch covers a head and a tail around a whole-line run.
  uint64_t skip_at = ~0ull;
  uint64_t skip = 0;
};

// ---------------------------------------------------------------------------------
// Uniform kernel, LDS-DMA form.  Same arithmetic as the register kernels, but each
// slot's 1 KiB (64 lanes x 16 B) arrives through global_load_lds_dwordx4 into a
// per-wave ring of kDmaRing LDS slots instead of VGPRs:
//     wait for slot t -> ds_read_b128 -> DMA for slot t + kDmaRing into the same
//     LDS slot -> table lookups for slot t.
// kDmaRing KiB per wave, 16 waves: up to 80 KiB of reads in flight per CU, and the
// returning data never competes with the lookups for VGPR write ports (register
// rings lose bandwidth as per-slot VALU work grows).
//
// Waits.  hipcc drains vmcnt(0) before any LDS read it sees after an LDS-DMA, so the
// ring read is one asm statement: s_waitcnt vmcnt(kDmaRing-1) (every DMA completes in
// issue order and kDmaRing-1 DMAs are always issued after the one awaited; other
// vector-memory ops only make the wait stricter), ds_read_b128, lgkmcnt(0) (the read
// must retire before the slot is refilled).  The DMAs themselves are unconditional
// (lanes past the end re-read the batch's last packet), so the count never drifts.
//
// Results of 8 rounds are collected in one register (lane 8g+j = round j's packet of
// group g) and written by one store.  The whole batch goes through this kernel:
// slot-0 chunks that lie wholly before their packet read the zero chunk; the one lane
// whose slot-0 chunk straddles the packet start reads the straddled words with
// load_top_words only when the chunk would reach below the caller's base.
// ---------------------------------------------------------------------------------
typedef __attribute__((address_space(3))) void LdsVoid;
typedef __attribute__((address_space(3))) char LdsChar;
constexpr int kUniformRing = 5;                              // LDS slots per wave, uniform kernel
constexpr uint32_t kRingStride = kWavesPerBlock * 64 * 16;   // bytes between ring positions

// All LDS of a DMA kernel in ONE variable, tables first: the fused asm lookups use
// raw LDS addresses and need the tables at address 0 (checked at kernel start).
template <int R>
struct UniformDmaLds {
  uint32_t tables[kLdsDwords];
  u32x4 ring[R][kWavesPerBlock][64];
  uint32_t next_dispatch;
};
static_assert(sizeof(UniformDmaLds<kUniformRing>) <= 160 * 1024, "LDS");

// Wait until at most N DMAs are outstanding, read the landed slot (16 B per lane),
// and wait for the read (the slot is refilled right after).
template <int N>
__device__ __forceinline__ u32x4 read_landed_slot(uint32_t addr) {
  u32x4 v;
  asm volatile(
      "s_waitcnt vmcnt(%1)\n\t"
      "ds_read_b128 %0, %2\n\t"
      "s_waitcnt lgkmcnt(0)"
      : "=v"(v)
      : "i"(N), "v"(addr)
      : "memory");
  return v;
}

// One Horner step on 4 words fused with the next slot's ring read, so a slot costs one
// LDS round trip instead of three: the 16 table lookups are issued, then the wait for
// the next slot's DMA (vmcnt(N)) and its ds_read_b128, then a single lgkmcnt(0) and
// the XORs.  One asm statement: the compiler never sees a pending LDS result.  The
// main tables must start at LDS address 0 (checked at the kernel's start).
template <int N>
__device__ __forceinline__ void horner_step_and_read(const Lookup& lk, uint32_t& h0, uint32_t& h1, uint32_t& h2,
                                                     uint32_t& h3, uint32_t w0, uint32_t w1, uint32_t w2,
                                                     uint32_t w3, uint32_t next_addr, u32x4& next) {
  uint32_t a[16];
  const uint32_t hs[4] = {h0, h1, h2, h3};
#pragma unroll
  for (int j = 0; j < 4; ++j) {
#pragma unroll
    for (int t = 0; t < 4; ++t) a[4 * j + t] = lookup_addr(hs[j], lk.lp, lk, t);
  }
  asm volatile(
      "ds_read_b32 %5, %5\n\tds_read_b32 %6, %6\n\tds_read_b32 %7, %7\n\tds_read_b32 %8, %8\n\t"
      "ds_read_b32 %9, %9\n\tds_read_b32 %10, %10\n\tds_read_b32 %11, %11\n\tds_read_b32 %12, %12\n\t"
      "ds_read_b32 %13, %13\n\tds_read_b32 %14, %14\n\tds_read_b32 %15, %15\n\tds_read_b32 %16, %16\n\t"
      "ds_read_b32 %17, %17\n\tds_read_b32 %18, %18\n\tds_read_b32 %19, %19\n\tds_read_b32 %20, %20\n\t"
      "s_waitcnt vmcnt(%26)\n\t"
      "ds_read_b128 %4, %21\n\t"
      "s_waitcnt lgkmcnt(0)\n\t"
      "v_bitop3_b32 %5, %5, %6, %7 bitop3:0x96\n\t"
      "v_bitop3_b32 %0, %5, %8, %22 bitop3:0x96\n\t"
      "v_bitop3_b32 %9, %9, %10, %11 bitop3:0x96\n\t"
      "v_bitop3_b32 %1, %9, %12, %23 bitop3:0x96\n\t"
      "v_bitop3_b32 %13, %13, %14, %15 bitop3:0x96\n\t"
      "v_bitop3_b32 %2, %13, %16, %24 bitop3:0x96\n\t"
      "v_bitop3_b32 %17, %17, %18, %19 bitop3:0x96\n\t"
      "v_bitop3_b32 %3, %17, %20, %25 bitop3:0x96"
      : "=&v"(h0), "=&v"(h1), "=&v"(h2), "=&v"(h3), "=&v"(next), "+v"(a[0]), "+v"(a[1]), "+v"(a[2]),
        "+v"(a[3]), "+v"(a[4]), "+v"(a[5]), "+v"(a[6]), "+v"(a[7]), "+v"(a[8]), "+v"(a[9]), "+v"(a[10]),
        "+v"(a[11]), "+v"(a[12]), "+v"(a[13]), "+v"(a[14]), "+v"(a[15])
      : "v"(next_addr), "v"(w0), "v"(w1), "v"(w2), "v"(w3), "i"(N)
      : "memory");
}

// LDS atomic add in asm: hipcc would otherwise order it behind every in-flight LDS-DMA
// (it cannot tell the counter from the ring) and drain the ring with vmcnt(0).
__device__ __forceinline__ uint32_t lds_fetch_add_one(uint32_t* counter) {
  uint32_t old;
  const uint32_t addr = (uint32_t)(uintptr_t)(LdsVoid*)counter, one = 1;
  asm volatile(
      "ds_add_rtn_u32 %0, %1, %2\n\t"
      "s_waitcnt lgkmcnt(0)"
      : "=v"(old)
      : "v"(addr), "v"(one)
      : "memory");
  return old;
}

// Work distribution.  Workgroup b owns the rounds b*16 + j + i*16*gridDim (j < 16),
// i.e. the whole grid sweeps the batch front to back together.  Inside the workgroup
// the waves take those rounds in order from an LDS counter instead of statically:
// the SIMD arbiter favours older waves, and with a static split the youngest waves of
// a CU finished up to 1.5x later than the oldest, leaving the CU
// half-occupied at the end.  A wave knows its next kLook rounds ahead of time (the
// ring prefetches that far) and fetches one more per round.
// Packets of 15 steps and more (1793 B .. 4 KiB; shorter ones take the register ring,
// longer ones the wave-per-packet kernel); runtime step count.
//
// Trailing bytes: every packet is run to the next 4-byte boundary (Lx = length
// rounded up), the z = Lx - length bytes past its end are masked to zero in the last
// word (lane 0's last slot), and the combine's last-word shift stops z bytes short
// (finish_word).  No separate tail-word load.
//
// kNT: the DMAs carry the non-temporal hint.  Only for batches whose packets all END on
// a 128-B line (launch_uniform): then every slot of a group is one whole aligned line,
// never shared with a neighbour, and streaming whole lines past the caches is what the
// memory system does fastest (tools/dma_probe PROBE_LINES: 8 aligned lines per
// instruction with the kernel's lookups, 197 us non-temporal vs 219.5 us plain for
// 1.26 GB; on lines a packet shares with its neighbour the hint costs a second fetch).
template <bool kNT>
__global__ __launch_bounds__(kBlock) void crc32_uniform_dma_kernel(UniformBatch u, uint32_t* __restrict__ out) {
  send_servers_home();
  constexpr int kDmaRing = kUniformRing;
  __shared__ __attribute__((aligned(16))) UniformDmaLds<kDmaRing> S;
  uint32_t* const lds = S.tables;
  auto& ring = S.ring;
  uint32_t& next_dispatch = S.next_dispatch;
  constexpr int kLook = 2;  // rounds a wave must know ahead
  if (threadIdx.x == 0) next_dispatch = kWavesPerBlock * kLook;
  fill_lds(lds);
  __syncthreads();
  const LaneConsts c = lane_consts(u.base);
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);

  const uint64_t total_rounds = (u.count + kPacketsPerWave - 1) / kPacketsPerWave;
  const uint64_t sweep = (uint64_t)gridDim.x * kWavesPerBlock;
  auto round_of = [&](uint32_t d) -> uint64_t {
    return (uint64_t)blockIdx.x * kWavesPerBlock + (d % kWavesPerBlock) + (uint64_t)(d / kWavesPerBlock) * sweep;
  };

  const uint32_t lx = (u.length + 3u) & ~3u, z = lx - u.length;
  const PacketGeo g = make_geo(0, lx);
  const int32_t ns = g.nsteps;  // >= kDmaRing (launch_uniform)
  const uint32_t last_mask = c.k == 0 ? 0xFFFFFFFFu >> (8u * z) : 0xFFFFFFFFu;  // lane 0 holds the last word
  // This lane's slot-0 chunk relative to its packet's start (> -128: DESIGN.md §3).
  const int64_t rel0 = (int64_t)g.a1 - 16 * (int64_t)(c.k + 1u) - (int64_t)kBytesPerStep * (ns - 1);
  uint32_t am[4], xm[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    am[j] = rel0 + 4 * j >= 0 ? 0xFFFFFFFFu : 0u;
    xm[j] = rel0 + 4 * j == 0 ? kInitRegister : 0u;
  }
  const bool none0 = rel0 <= -16;             // slot-0 chunk wholly before the packet
  const bool part0 = rel0 < 0 && rel0 > -16;  // straddles the packet start
  const uint32_t head_meta = part0 ? (uint32_t)(rel0 / 4 + 4) : 0u;  // round_meta()'s head field

  // Packet of group `grp` in round `rnd`; rounds past the end re-read the last packet.
  auto packet_index = [&](uint64_t rnd, uint32_t grp) -> uint64_t {
    const uint64_t p = rnd * kPacketsPerWave + grp;
    return p < u.count ? p : u.count - 1;
  };
  auto packet_base = [&](uint64_t rnd) -> uint64_t { return u.base + packet_index(rnd, c.grp) * u.stride; };
  auto is_below = [&](uint64_t pb) -> bool { return part0 && (int64_t)(pb - u.base) + rel0 < 0; };
  auto slot_src = [&](uint64_t pb, int32_t s) -> uint64_t {
    if (s != 0) return pb + (uint64_t)(rel0 + (int64_t)kBytesPerStep * s);
    return none0 || is_below(pb) ? c.dummy : pb + (uint64_t)rel0;
  };
  // LDS byte address of ring position 0 for this wave; DMA destinations are wave-uniform.
  const uint32_t ring0 = (uint32_t)(uintptr_t)(LdsVoid*)&ring[0][wv][0];
  auto dma = [&](uint64_t src, uint32_t q) {
    __builtin_amdgcn_global_load_lds((const void*)src, (LdsVoid*)&ring[q][wv][0], 16, 0, kNT ? 2 : 0);
  };

  uint64_t rnd[kLook + 1];  // rnd[0]: current round; rnd[i]: i rounds ahead (wave-uniform)
#pragma unroll
  for (int i = 0; i < kLook; ++i) rnd[i] = round_of(wv + (uint32_t)(kWavesPerBlock * i));
  if (rnd[0] >= total_rounds) return;
  if ((uint32_t)(uintptr_t)(LdsVoid*)lds != 0) __builtin_trap();  // horner_step_and_read addresses
#pragma unroll
  for (int f = 0; f < kDmaRing; ++f) dma(slot_src(packet_base(rnd[0]), f), (uint32_t)f);  // ns >= kDmaRing
  uint32_t q = 0;  // ring position of the slot being consumed (wave-uniform)
  // The ring is read one slot ahead: `nextv` holds the slot about to be consumed.
  u32x4 nextv = read_landed_slot<kDmaRing - 1>(ring0 + lane * 16u);
  uint32_t res = 0, j = 0;
  uint64_t res_round = 0;
  while (rnd[0] < total_rounds) {
    // Claim the round kLook ahead; its index is first needed one round from now.
    uint32_t d = 0;
    if (lane == 0) d = lds_fetch_add_one(&next_dispatch);
    const uint64_t pb = packet_base(rnd[0]);
    const uint64_t pb_next = packet_base(rnd[1]);
    uint32_t h0 = 0, h1 = 0, h2 = 0, h3 = 0;
    // One slot: wait for it, refill its LDS slot kDmaRing slots ahead, then the lookups.
    auto slot = [&](int32_t s, bool top, bool last) {
      const u32x4 v = nextv;
      const int32_t f = s + kDmaRing;  // refill this slot's LDS slot kDmaRing slots ahead
      dma(f < ns ? slot_src(pb, f) : slot_src(pb_next, f - ns), q);
      q = q + 1 == (uint32_t)kDmaRing ? 0u : q + 1;
      const uint32_t next_addr = ring0 + q * kRingStride + lane * 16u;
      uint32_t w0 = v.x, w1 = v.y, w2 = v.z, w3 = v.w;
      if (top) {
        const bool below = is_below(pb);
        if (__builtin_amdgcn_ballot_w64(below)) {
          if (below) load_top_words(pb + (uint64_t)rel0, head_meta, c.dummy, w0, w1, w2, w3);
        }
      }
      if (last) w3 &= last_mask;  // data only: before the initial-register injection below
      if (top) {  // top step: M32^32(0) = 0, no lookups; mask to the packet's bytes
        h0 = (w0 & am[0]) ^ xm[0];
        h1 = (w1 & am[1]) ^ xm[1];
        h2 = (w2 & am[2]) ^ xm[2];
        h3 = (w3 & am[3]) ^ xm[3];
        nextv = read_landed_slot<kDmaRing - 1>(next_addr);
      } else {
        horner_step_and_read<kDmaRing - 1>(c.lk, h0, h1, h2, h3, w0, w1, w2, w3, next_addr, nextv);
      }
      issue_order_fence();  // keep each slot's lookups between its DMA and the next slot's wait
    };
    slot(0, true, false);  // ns >= kDmaRing > 1
    for (int32_t s = 1; s < ns - 1; ++s) slot(s, false, false);
    slot(ns - 1, false, true);
    const uint32_t y = combine_tree(lds, h0, h1, h2, h3, c.lk);
    uint32_t reg = finish_word(lds, y, z, c.lk);  // every lane; lane k == 0 holds the register
    const uint32_t crc = (uint32_t)__shfl((int)__builtin_bswap32(~reg), (int)(lane & ~7u), 64);
    // Lane 8g+j keeps the checksum of group g in this wave's j-th round of 8; one store per 8.
    if (c.k == j) {
      res = crc;
      res_round = rnd[0];
    }
#pragma unroll
    for (int i = 0; i < kLook - 1; ++i) rnd[i] = rnd[i + 1];
    rnd[kLook - 1] = round_of(__builtin_amdgcn_readfirstlane(d));
    if (j == 7u || rnd[0] >= total_rounds) {
      const uint64_t p = res_round * kPacketsPerWave + c.grp;
      if (c.k <= j && p < u.count) out[p] = res;
      j = 0;
    } else {
      ++j;
    }
  }
  // The ring's last DMAs (re-reads of valid packets) must land before the wave's LDS goes away.
  __builtin_amdgcn_s_waitcnt(0);
}

// ---------------------------------------------------------------------------------
// Wave-per-packet kernel for long uniform packets (from 4 KiB; packets of a multiple of 8 KiB
// steps take the register-ring form crc32_wave_regs_kernel below): the whole wave
// works on ONE packet and each step is one KiB of it, lane l taking the 16-B chunk
// at a1 - 16 (l + 1) - 1024 (ns - 1 - s).  So every DMA instruction reads 1 KiB of
// contiguous bytes (8 consecutive 128-B lines) instead of one line from each of 8
// packets, the shape the read probes stream fastest with the non-temporal hint
// (tools/dma_probe: whole contiguous KiB 193-199 us for 1.26 GB).
// Arithmetic: the same 4 word streams per lane, with the Horner operator M32^256 (a
// 1-KiB stride) in the replicated block's main set; at the packet's end the in-lane
// M32^1 combine, then a 6-level tree over the 64 lanes (M32^4 .. M32^128; DPP inside
// 16-lane rows, shuffles for the last two levels) and finish_word on lane 0.
// Same LDS-DMA ring, waits, head/tail masking and dispatch as crc32_uniform_dma_kernel
// (a "round" is one packet here).  Packets of >= kWaveRing KiB only.
// ---------------------------------------------------------------------------------
constexpr int kWaveRing = 4;
constexpr uint32_t kWaveStep = 1024;
constexpr int kWaveTreeLevels = 6;
constexpr uint32_t kWaveTreeDword = kRepDwords;
constexpr uint32_t kWaveLdsDwords = kWaveTreeDword + kWaveTreeLevels * 1024;
static_assert(kMainLevel + 3 < kOpLevels, "M32^256 table level");

struct WaveDmaLds {
  uint32_t tables[kWaveLdsDwords];
  u32x4 ring[kWaveRing][kWavesPerBlock][64];
  uint32_t next_dispatch;
};
static_assert(sizeof(WaveDmaLds) <= 160 * 1024, "LDS");

__device__ __forceinline__ void fill_lds_wave(uint32_t* lds) {
  store_tables<kWaveTreeLevels>(lds, kWaveTreeDword, load_tables<kWaveTreeLevels>(kMainLevel + 3, 0));
}

// The packet's register before the shift of its last word (register = M32 y), valid
// on lane 0: in-lane Horner over the 4 word slots, then lane l + d folds into lane l
// through M32^(4d) for d = 1, 2, 4, ..., 32.
__device__ __forceinline__ uint32_t combine_wave(const uint32_t* lds, uint32_t h0, uint32_t h1, uint32_t h2,
                                                uint32_t h3, const Lookup& lk) {
  uint32_t y = apply_rep(lds, h0, h1, lk.lp1, lk);
  y = apply_rep(lds, y, h2, lk.lp1, lk);
  y = apply_rep(lds, y, h3, lk.lp1, lk);
  const uint32_t l = threadIdx.x & 63u;
  const uint32_t* tree = lds + kWaveTreeDword;
  uint32_t t = 0;
  if (l & 1u) t = apply_small(tree, y);
  y ^= from_lane_plus<1>(t);
  if ((l & 3u) == 2u) t = apply_small(tree + 1024, y);
  y ^= from_lane_plus<2>(t);
  if ((l & 7u) == 4u) t = apply_small(tree + 2048, y);
  y ^= from_lane_plus<4>(t);
  if ((l & 15u) == 8u) t = apply_small(tree + 3072, y);
  y ^= from_lane_plus<8>(t);
  if ((l & 31u) == 16u) t = apply_small(tree + 4096, y);
  y ^= (uint32_t)__shfl((int)t, (int)((l + 16u) & 63u), 64);
  if (l == 32u) t = apply_small(tree + 5120, y);
  y ^= (uint32_t)__shfl((int)t, (int)((l + 32u) & 63u), 64);
  return y;
}

template <bool kNT>
__global__ __launch_bounds__(kBlock) void crc32_wave_dma_kernel(UniformBatch u, uint32_t* __restrict__ out) {
  send_servers_home();
  constexpr int kDmaRing = kWaveRing;
  __shared__ __attribute__((aligned(16))) WaveDmaLds S;
  uint32_t* const lds = S.tables;
  auto& ring = S.ring;
  uint32_t& next_dispatch = S.next_dispatch;
  constexpr int kLook = 2;
  if (threadIdx.x == 0) next_dispatch = kWavesPerBlock * kLook;
  fill_lds_wave(lds);
  __syncthreads();
  const LaneConsts c = lane_consts(u.base);
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint64_t total = u.count;
  const uint64_t sweep = (uint64_t)gridDim.x * kWavesPerBlock;
  auto round_of = [&](uint32_t d) -> uint64_t {
    return (uint64_t)blockIdx.x * kWavesPerBlock + (d % kWavesPerBlock) + (uint64_t)(d / kWavesPerBlock) * sweep;
  };
  const uint32_t lx = (u.length + 3u) & ~3u, z = lx - u.length;
  const int32_t ns = (int32_t)((lx + kWaveStep - 1) / kWaveStep);  // >= kDmaRing (launch_uniform)
  const uint32_t last_mask = lane == 0 ? 0xFFFFFFFFu >> (8u * z) : 0xFFFFFFFFu;
  // This lane's step-0 chunk relative to its packet's start (> -1024).
  const int64_t rel0 = (int64_t)lx - 16 * (int64_t)(lane + 1u) - (int64_t)kWaveStep * (ns - 1);
  uint32_t am[4], xm[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    am[j] = rel0 + 4 * j >= 0 ? 0xFFFFFFFFu : 0u;
    xm[j] = rel0 + 4 * j == 0 ? kInitRegister : 0u;
  }
  const bool none0 = rel0 <= -16;
  const bool part0 = rel0 < 0 && rel0 > -16;
  const uint32_t head_meta = part0 ? (uint32_t)(rel0 / 4 + 4) : 0u;
  auto packet_base = [&](uint64_t p) -> uint64_t { return u.base + (p < total ? p : total - 1) * u.stride; };
  auto is_below = [&](uint64_t pb) -> bool { return part0 && (int64_t)(pb - u.base) + rel0 < 0; };
  auto slot_src = [&](uint64_t pb, int32_t s) -> uint64_t {
    if (s != 0) return pb + (uint64_t)(rel0 + (int64_t)kWaveStep * s);
    return none0 || is_below(pb) ? c.dummy : pb + (uint64_t)rel0;
  };
  const uint32_t ring0 = (uint32_t)(uintptr_t)(LdsVoid*)&ring[0][wv][0];
  auto dma = [&](uint64_t src, uint32_t q) {
    __builtin_amdgcn_global_load_lds((const void*)src, (LdsVoid*)&ring[q][wv][0], 16, 0, kNT ? 2 : 0);
  };

  uint64_t rnd0 = round_of(wv), rnd1 = round_of(wv + kWavesPerBlock);
  if (rnd0 >= total) return;
  if ((uint32_t)(uintptr_t)(LdsVoid*)lds != 0) __builtin_trap();  // horner_step_and_read addresses
#pragma unroll
  for (int f = 0; f < kDmaRing; ++f) dma(slot_src(packet_base(rnd0), f), (uint32_t)f);
  uint32_t q = 0;
  u32x4 nextv = read_landed_slot<kDmaRing - 1>(ring0 + lane * 16u);
  while (rnd0 < total) {
    uint32_t d = 0;
    if (lane == 0) d = lds_fetch_add_one(&next_dispatch);
    const uint64_t pb = packet_base(rnd0), pb_next = packet_base(rnd1);
    uint32_t h0 = 0, h1 = 0, h2 = 0, h3 = 0;
    auto slot = [&](int32_t s, bool top, bool last) {
      const u32x4 v = nextv;
      const int32_t f = s + kDmaRing;
      dma(f < ns ? slot_src(pb, f) : slot_src(pb_next, f - ns), q);
      q = q + 1 == (uint32_t)kDmaRing ? 0u : q + 1;
      const uint32_t next_addr = ring0 + q * kRingStride + lane * 16u;
      uint32_t w0 = v.x, w1 = v.y, w2 = v.z, w3 = v.w;
      if (top) {
        const bool below = is_below(pb);
        if (__builtin_amdgcn_ballot_w64(below)) {
          if (below) load_top_words(pb + (uint64_t)rel0, head_meta, c.dummy, w0, w1, w2, w3);
        }
      }
      if (last) w3 &= last_mask;
      if (top) {
        h0 = (w0 & am[0]) ^ xm[0];
        h1 = (w1 & am[1]) ^ xm[1];
        h2 = (w2 & am[2]) ^ xm[2];
        h3 = (w3 & am[3]) ^ xm[3];
        nextv = read_landed_slot<kDmaRing - 1>(next_addr);
      } else {
        horner_step_and_read<kDmaRing - 1>(c.lk, h0, h1, h2, h3, w0, w1, w2, w3, next_addr, nextv);
      }
      issue_order_fence();
    };
    slot(0, true, false);  // ns >= kDmaRing > 1
    for (int32_t s = 1; s < ns - 1; ++s) slot(s, false, false);
    slot(ns - 1, false, true);
    const uint32_t y = combine_wave(lds, h0, h1, h2, h3, c.lk);
    const uint32_t reg = finish_word(lds, y, z, c.lk);  // lane 0 holds the register
    if (lane == 0) out[rnd0] = __builtin_bswap32(~reg);
    rnd0 = rnd1;
    rnd1 = round_of(__builtin_amdgcn_readfirstlane(d));
  }
  __builtin_amdgcn_s_waitcnt(0);
}

// crc32_wave_dma_kernel with the slots in a register ring of kWaveRegRing KiB per wave
// (non-temporal global loads when kNT) instead of the LDS-DMA ring, for packets of a multiple
// of kWaveRegRing KiB steps (the 64-KiB buffers of configs[4]): 327-329 us vs 334-339 us for
// 32,768 x 64 KiB, 4 alternating pairs (profiles/r03/waveregs).  Same arithmetic, masks,
// dispatch and combine; the next packet's first kWaveRegRing steps load during the last ones.
constexpr int kWaveRegRing = 8;
typedef __attribute__((address_space(1))) const u32x4 GlobalU32x4W;

template <bool kNT>
__global__ __launch_bounds__(kBlock) void crc32_wave_regs_kernel(UniformBatch u, uint32_t* __restrict__ out) {
  send_servers_home();
  constexpr int D = kWaveRegRing;
  __shared__ __attribute__((aligned(16))) WaveDmaLds S;
  uint32_t* const lds = S.tables;
  if (threadIdx.x == 0) S.next_dispatch = kWavesPerBlock * 2;
  fill_lds_wave(lds);
  __syncthreads();
  const LaneConsts c = lane_consts(u.base);
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint64_t total = u.count;
  const uint64_t sweep = (uint64_t)gridDim.x * kWavesPerBlock;
  auto round_of = [&](uint32_t d) -> uint64_t {
    return (uint64_t)blockIdx.x * kWavesPerBlock + (d % kWavesPerBlock) + (uint64_t)(d / kWavesPerBlock) * sweep;
  };
  const uint32_t lx = (u.length + 3u) & ~3u, z = lx - u.length;
  const int32_t ns = (int32_t)((lx + kWaveStep - 1) / kWaveStep);  // a multiple of D (launch_uniform)
  const uint32_t last_mask = lane == 0 ? 0xFFFFFFFFu >> (8u * z) : 0xFFFFFFFFu;
  const int64_t rel0 = (int64_t)lx - 16 * (int64_t)(lane + 1u) - (int64_t)kWaveStep * (ns - 1);
  uint32_t am[4], xm[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    am[j] = rel0 + 4 * j >= 0 ? 0xFFFFFFFFu : 0u;
    xm[j] = rel0 + 4 * j == 0 ? kInitRegister : 0u;
  }
  const bool none0 = rel0 <= -16;
  const bool part0 = rel0 < 0 && rel0 > -16;
  const uint32_t head_meta = part0 ? (uint32_t)(rel0 / 4 + 4) : 0u;
  auto packet_base = [&](uint64_t p) -> uint64_t { return u.base + (p < total ? p : total - 1) * u.stride; };
  auto is_below = [&](uint64_t pb) -> bool { return part0 && (int64_t)(pb - u.base) + rel0 < 0; };
  auto slot_src = [&](uint64_t pb, int32_t s) -> uint64_t {
    if (s != 0) return pb + (uint64_t)(rel0 + (int64_t)kWaveStep * s);
    return none0 || is_below(pb) ? c.dummy : pb + (uint64_t)rel0;
  };
  auto ld = [&](uint64_t a) -> u32x4 {
    // kNT: every packet ends on a 128-B line, so each chunk is 16-B aligned; otherwise
    // chunks are only 4-B aligned (a base at +4 or +12): the packed 4-B-aligned type.
    if constexpr (kNT) return __builtin_nontemporal_load(reinterpret_cast<GlobalU32x4W*>(a));
    return load_chunk(a);
  };
  uint64_t rnd0 = round_of(wv), rnd1 = round_of(wv + kWavesPerBlock);
  if (rnd0 >= total) return;
  u32x4 q[D];
  {
    const uint64_t pb = packet_base(rnd0);
#pragma unroll
    for (int i = 0; i < D; ++i) {
      q[i] = ld(slot_src(pb, i));
      issue_order_fence();
    }
  }
  const int32_t iters = ns / D;
  while (rnd0 < total) {
    uint32_t d = 0;
    if (lane == 0) d = atomicAdd(&S.next_dispatch, 1u);
    const uint64_t pb = packet_base(rnd0), pbn = packet_base(rnd1);
    uint32_t h0 = 0, h1 = 0, h2 = 0, h3 = 0;
    for (int32_t it = 0; it < iters; ++it) {
      const bool first = it == 0, last = it == iters - 1;
#pragma unroll
      for (int i = 0; i < D; ++i) {
        uint32_t w0 = q[i].x, w1 = q[i].y, w2 = q[i].z, w3 = q[i].w;
        if (i == 0 && first) {
          const bool below = is_below(pb);
          if (__builtin_amdgcn_ballot_w64(below)) {
            if (below) load_top_words(pb + (uint64_t)rel0, head_meta, c.dummy, w0, w1, w2, w3);
          }
        }
        if (i == D - 1 && last) w3 &= last_mask;
        if (i == 0 && first) {
          h0 = (w0 & am[0]) ^ xm[0];
          h1 = (w1 & am[1]) ^ xm[1];
          h2 = (w2 & am[2]) ^ xm[2];
          h3 = (w3 & am[3]) ^ xm[3];
        } else {
          h0 = horner_main(lds, h0, w0, c.lk);
          h1 = horner_main(lds, h1, w1, c.lk);
          h2 = horner_main(lds, h2, w2, c.lk);
          h3 = horner_main(lds, h3, w3, c.lk);
        }
        issue_order_fence();
        q[i] = ld(last ? slot_src(pbn, i) : slot_src(pb, (it + 1) * D + i));
        issue_order_fence();
      }
    }
    const uint32_t y = combine_wave(lds, h0, h1, h2, h3, c.lk);
    const uint32_t reg = finish_word(lds, y, z, c.lk);
    if (lane == 0) out[rnd0] = __builtin_bswap32(~reg);
    rnd0 = rnd1;
    rnd1 = round_of(__builtin_amdgcn_readfirstlane(d));
  }
}

// ---------------------------------------------------------------------------------
// Uniform kernel, register form: the G1 path (packets of 1..14 steps, <= 1792 B).  Same
// geometry, arithmetic, dispatch, result batching and trailing-byte handling as
// crc32_uniform_dma_kernel, but the packet bytes go straight to VGPRs: the next round's
// chunks are loaded into the ring registers while this round's are consumed (NS + 1
// KiB per wave in flight) and LDS serves only the table lookups (no DMA write, no ring
// read).  Every load is unconditional and issued in slot order, so hipcc's waitcnts
// stay exact.
//
// Line-split loads: the ring has NS + 1 entries and each load reads, per group,
// the chunks of ONE 128-B line (aligned to the packet end's 16-B residue) instead of one
// end-aligned 128-B piece, which straddles two lines.  A piece i of the packet (end at
// a1, j = (a1 mod 128) / 16) is the top 8 - j chunks of one line plus the bottom j of the
// next, so lane k finds its slot-s chunk in entry s + lo, lo = (k < j): entry u holds
// lane k's slot u - lo chunk (slots -1 and NS read the zero chunk).  Same bytes, same
// lookups; one more load per round, but 8 whole lines per load instruction instead of
// 16 partial ones (tools/dma_probe PROBE_SPLIT: 217-219 us vs 224-229 us for the piece
// loads, same box, alternating).
// ---------------------------------------------------------------------------------
// The whole-line kernel's LDS: the ragged kernel's table layout (the replicated main block and the
// unreplicated tree sets that tree_levels_asm reads), 76 KiB instead of the register kernels' 132.
struct UniformLinesLds {
  uint32_t tables[kLdsDwords];
  uint32_t next_dispatch;
};
struct UniformRegsLds {
  uint32_t tables[kRegsLdsDwords];
  uint32_t next_dispatch;
};

template <int NS>
__global__ __launch_bounds__(kBlock) void crc32_uniform_regs_kernel(UniformBatch u, uint32_t* __restrict__ out) {
  send_servers_home();
  __shared__ __attribute__((aligned(16))) UniformRegsLds S;
  uint32_t* const lds = S.tables;
  if (threadIdx.x == 0) S.next_dispatch = kWavesPerBlock * 2;
  fill_lds_regs(lds);
  __syncthreads();
  const LaneConsts c = lane_consts(u.base);
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);

  const uint64_t total_rounds = (u.count + kPacketsPerWave - 1) / kPacketsPerWave;
  const uint64_t sweep = (uint64_t)gridDim.x * kWavesPerBlock;
  auto round_of = [&](uint32_t d) -> uint64_t {
    return (uint64_t)blockIdx.x * kWavesPerBlock + (d % kWavesPerBlock) + (uint64_t)(d / kWavesPerBlock) * sweep;
  };
  const uint32_t lx = (u.length + 3u) & ~3u, z = lx - u.length;
  const PacketGeo g = make_geo(0, lx);
  const uint32_t last_mask = c.k == 0 ? 0xFFFFFFFFu >> (8u * z) : 0xFFFFFFFFu;
  const int64_t rel0 = (int64_t)g.a1 - 16 * (int64_t)(c.k + 1u) - (int64_t)kBytesPerStep * (NS - 1);
  uint32_t am[4], xm[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    am[j] = rel0 + 4 * j >= 0 ? 0xFFFFFFFFu : 0u;
    xm[j] = rel0 + 4 * j == 0 ? kInitRegister : 0u;
  }
  const bool none0 = rel0 <= -16;
  const bool part0 = rel0 < 0 && rel0 > -16;
  const uint32_t head_meta = part0 ? (uint32_t)(rel0 / 4 + 4) : 0u;
  auto batch_index = [&](uint64_t p) -> uint64_t { return p + (p >= u.skip_at ? u.skip : 0u); };
  auto packet_base = [&](uint64_t rnd) -> uint64_t {
    const uint64_t p = rnd * kPacketsPerWave + c.grp;
    return u.base + batch_index(p < u.count ? p : u.count - 1) * u.stride;
  };
  auto is_below = [&](uint64_t pb) -> bool { return part0 && (int64_t)(pb - u.base) + rel0 < 0; };
  auto slot_src = [&](uint64_t pb, int32_t s) -> uint64_t {
    if (s != 0) return pb + (uint64_t)(rel0 + (int64_t)kBytesPerStep * s);
    return none0 || is_below(pb) ? c.dummy : pb + (uint64_t)rel0;
  };

  uint64_t rnd0 = round_of(wv), rnd1 = round_of(wv + kWavesPerBlock);
  if (rnd0 >= total_rounds) return;
  constexpr int NE = NS + 1;  // ring entries
  // Ring entry e of the round whose packet (this group's) starts at pb.
  auto entry_src = [&](uint64_t pb, int e) -> uint64_t {
    const uint32_t lo = c.k < ((uint32_t)(pb + lx) & 127u) >> 4 ? 1u : 0u;
    const int32_t sl = e - (int32_t)lo;
    return sl < 0 || sl >= NS ? c.dummy : slot_src(pb, sl);
  };
  u32x4 q[NE];
  {
    const uint64_t pb = packet_base(rnd0);
#pragma unroll
    for (int e = 0; e < NE; ++e) {
      q[e] = load_chunk(entry_src(pb, e));
      issue_order_fence();
    }
  }
  uint32_t res = 0, j = 0;
  uint64_t res_round = 0;
  while (rnd0 < total_rounds) {
    uint32_t d = 0;
    if (lane == 0) d = atomicAdd(&S.next_dispatch, 1u);
    const uint64_t pb = packet_base(rnd0), pbn = packet_base(rnd1);
    const bool lo = c.k < (((uint32_t)(pb + lx) & 127u) >> 4);
    uint32_t h0 = 0, h1 = 0, h2 = 0, h3 = 0;
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      const u32x4 v = lo ? q[s + 1] : q[s];
      uint32_t w0 = v.x, w1 = v.y, w2 = v.z, w3 = v.w;
      if (s == 0) {
        const bool below = is_below(pb);
        if (__builtin_amdgcn_ballot_w64(below)) {
          if (below) load_top_words(pb + (uint64_t)rel0, head_meta, c.dummy, w0, w1, w2, w3);
        }
      }
      if (s == NS - 1) w3 &= last_mask;
      if (s == 0) {
        h0 = (w0 & am[0]) ^ xm[0];
        h1 = (w1 & am[1]) ^ xm[1];
        h2 = (w2 & am[2]) ^ xm[2];
        h3 = (w3 & am[3]) ^ xm[3];
      } else {
        h0 = horner_main(lds, h0, w0, c.lk);
        h1 = horner_main(lds, h1, w1, c.lk);
        h2 = horner_main(lds, h2, w2, c.lk);
        h3 = horner_main(lds, h3, w3, c.lk);
      }
      issue_order_fence();
      q[s] = load_chunk(entry_src(pbn, s));  // the next round's entry s
      issue_order_fence();
    }
    q[NS] = load_chunk(entry_src(pbn, NS));
    issue_order_fence();
    const uint32_t y = combine_tree_rep(lds, h0, h1, h2, h3, c.lk);
    uint32_t reg = finish_word(lds, y, z, c.lk);  // every lane; lane k == 0 holds the register
    const uint32_t crc = (uint32_t)__shfl((int)__builtin_bswap32(~reg), (int)(lane & ~7u), 64);
    if (c.k == j) {
      res = crc;
      res_round = rnd0;
    }
    rnd0 = rnd1;
    rnd1 = round_of(__builtin_amdgcn_readfirstlane(d));
    if (j == 7u || rnd0 >= total_rounds) {
      const uint64_t p = res_round * kPacketsPerWave + c.grp;
      if (c.k <= j && p < u.count) out[batch_index(p)] = res;
      j = 0;
    } else {
      ++j;
    }
  }
}

// ---------------------------------------------------------------------------------
// Uniform kernel, whole-line form (the G1 path): back-to-back packets (stride == length)
// whose length L is a multiple of 16 from a 128-B aligned base.  A round of 8 packets is
// then 8L bytes = a whole number of 128-B lines starting on a line, and group g reads the
// round's lines [Lg, Lg+1), Lg = floor(g L / 128): every line of the batch is read once,
// whole, by one non-temporal load (the non-temporal hint pays only on lines read once; on a
// line two packets share, the second read misses: tools/dma_probe P9).
//   * Lane k of group g reads chunk m = (j1 - 1 - k) mod 8 of each of its lines, where
//     j1 = ((g + 1) L mod 128) / 16 chunks of packet g lie in the next group's first line.
//     Then the lane holds position k (chunk index from the packet end, mod 8) of every
//     line, so the streams combine with the usual tree.  Slot s is line Lg+1 - NSL + s
//     (NSL = ceil(L / 128)); a group with one line fewer reads the zero chunk in slot 0.
//   * At the group's first line, chunks m < jg (jg = (g L mod 128) / 16) belong to packet
//     g - 1: they are zeroed in the stream and kept; chunk m == jg is packet g's first
//     (the initial register is XOR-ed into its first word).
//   * After the round's slots, lane k < j1 takes its step-0 chunk, which group g + 1 kept,
//     by ds_bpermute from lane (j2 - j1 + k) mod 8 of that group, and runs one more
//     Horner step (the other lanes' last chunk was slot NSL - 1).
// The launch covers count / 8 whole rounds; launch_uniform sends the < 8 packets left to
// the register kernel.  The lines stream through a register ring like
// crc32_uniform_regs_kernel's (the same lines through the LDS-DMA ring measured 3-5 % slower:
// profiles/r03/parked/lines_dma_ring_kernel.patch).
// ---------------------------------------------------------------------------------
typedef __attribute__((address_space(1))) const u32x4 GlobalU32x4;

template <int NSL>
__global__ __launch_bounds__(kBlock) void crc32_uniform_lines_kernel(UniformBatch u, uint32_t* __restrict__ out) {
  send_servers_home();
  __shared__ __attribute__((aligned(16))) UniformLinesLds S;
  uint32_t* const lds = S.tables;
  const LaneConsts c = lane_consts(u.base);
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint64_t rounds = u.count / kPacketsPerWave;
  const uint64_t sweep = (uint64_t)gridDim.x * kWavesPerBlock;
  auto round_of = [&](uint32_t d) -> uint64_t {
    return (uint64_t)blockIdx.x * kWavesPerBlock + (d % kWavesPerBlock) + (uint64_t)(d / kWavesPerBlock) * sweep;
  };
  const LinesLane ll = lines_lane(u.length, NSL, c.grp, c.k);
  const uint64_t round_bytes = (uint64_t)kPacketsPerWave * u.length;
  auto lane_base = [&](uint64_t rnd) -> uint64_t {
    return u.base + (rnd < rounds ? rnd : rounds - 1) * round_bytes + (uint64_t)ll.off0;
  };
  auto ld = [&](uint64_t lb, int s) -> u32x4 {
    const uint64_t a = s == 0 && ll.dummy0 ? c.dummy : lb + (uint64_t)kBytesPerStep * (uint64_t)s;
    return __builtin_nontemporal_load(reinterpret_cast<GlobalU32x4*>(a));
  };
  uint64_t rnd0 = round_of(wv), rnd1 = round_of(wv + kWavesPerBlock);
  u32x4 q[NSL];
  if (threadIdx.x == 0) S.next_dispatch = kWavesPerBlock * 2;
  // The table loads, then the first round's line loads (lane_base clamps a round past the
  // batch), then the table stores: the start pays one memory latency, not the table's and
  // then the first lines' in a row.
  const TableLoads<kTreeLevels> tl = load_tables<kTreeLevels>(kMainLevel, 0);
  issue_order_fence();
  {
    const uint64_t lb = lane_base(rnd0);
#pragma unroll
    for (int s = 0; s < NSL; ++s) {
      q[s] = ld(lb, s);
      issue_order_fence();
    }
  }
  store_tables<kTreeLevels>(lds, kTreeDword, tl);
  __syncthreads();
  if (rnd0 >= rounds) return;
  uint32_t res = 0, j = 0;
  uint64_t res_round = 0;
  uint32_t tree_a = 0x10000u;  // tree_levels_asm's address register (high half 1, kept)
  while (rnd0 < rounds) {
    uint32_t d = 0;
    if (lane == 0) d = atomicAdd(&S.next_dispatch, 1u);
    const uint64_t lbn = lane_base(rnd1);
    uint32_t h0 = 0, h1 = 0, h2 = 0, h3 = 0;
    u32x4 kept = {0u, 0u, 0u, 0u};
#pragma unroll
    for (int s = 0; s < NSL; ++s) {
      const u32x4 v = q[s];
      uint32_t w0 = v.x, w1 = v.y, w2 = v.z, w3 = v.w;
      if (s < 2) {
        if (ll.keep[s]) kept = v;
        w0 = (w0 & ll.am[s]) ^ ll.xm[s];
        w1 &= ll.am[s];
        w2 &= ll.am[s];
        w3 &= ll.am[s];
      }
      if (s == 0) {
        h0 = w0;
        h1 = w1;
        h2 = w2;
        h3 = w3;
      } else {
        h0 = horner_main(lds, h0, w0, c.lk);
        h1 = horner_main(lds, h1, w1, c.lk);
        h2 = horner_main(lds, h2, w2, c.lk);
        h3 = horner_main(lds, h3, w3, c.lk);
      }
      issue_order_fence();
      q[s] = ld(lbn, s);  // the next round's slot s
      issue_order_fence();
    }
    {
      const uint32_t a = ll.src4;
      const uint32_t x0 = (uint32_t)__builtin_amdgcn_ds_bpermute((int)a, (int)kept.x);
      const uint32_t x1 = (uint32_t)__builtin_amdgcn_ds_bpermute((int)a, (int)kept.y);
      const uint32_t x2 = (uint32_t)__builtin_amdgcn_ds_bpermute((int)a, (int)kept.z);
      const uint32_t x3 = (uint32_t)__builtin_amdgcn_ds_bpermute((int)a, (int)kept.w);
      const uint32_t s0 = horner_main(lds, h0, x0, c.lk), s1 = horner_main(lds, h1, x1, c.lk);
      const uint32_t s2 = horner_main(lds, h2, x2, c.lk), s3 = horner_main(lds, h3, x3, c.lk);
      h0 = ll.lo ? s0 : h0;
      h1 = ll.lo ? s1 : h1;
      h2 = ll.lo ? s2 : h2;
      h3 = ll.lo ? s3 : h3;
    }
    uint32_t y = apply_rep(lds, h0, h1, c.lk.lp1, c.lk);  // in-lane Horner over the 4 word streams
    y = apply_rep(lds, y, h2, c.lk.lp1, c.lk);
    y = apply_rep(lds, y, h3, c.lk.lp1, c.lk);
    y = tree_levels_asm(y, tree_a);
    const uint32_t reg = finish_word(lds, y, 0u, c.lk);
    const uint32_t crc = (uint32_t)__shfl((int)__builtin_bswap32(~reg), (int)(lane & ~7u), 64);
    if (c.k == j) {
      res = crc;
      res_round = rnd0;
    }
    rnd0 = rnd1;
    rnd1 = round_of(__builtin_amdgcn_readfirstlane(d));
    if (j == 7u || rnd0 >= rounds) {
      if (c.k <= j) out[res_round * kPacketsPerWave + c.grp] = res;
      j = 0;
    } else {
      ++j;
    }
  }
}

// ---------------------------------------------------------------------------------
// Ragged rounds on the LDS-DMA pair ring (crc32_ragged_jobs_kernel below).  Packets come
// sorted by step class, so the 8 packets of a round need (nearly) the same number of
// slots; a round runs NS = max(kPairMinSlots, max steps of its 8 rounded up to even) compute
// slots, loaded as NS / 2 pairs of 256 B per packet, and the packets with fewer steps read
// the zero chunk in their leading slots.  Per-round, per-lane geometry comes from each
// packet's record (round_from_record, pair_plan).  Trailing bytes as in the uniform DMA
// kernel: each packet runs to the next 4-byte boundary with the bytes past its end masked,
// then finish_word.
// ---------------------------------------------------------------------------------
// The DMA plan of one round for this lane: the address of its 16 B in pair 0 for each of its
// two DMA packets (the packet's end minus 128 NS, plus the lane's offset inside the 256-B
// pieces), and for each the first pair whose chunk of this lane is real (reaches the
// packet's top word and lies in the caller's buffer).  With t = the top word's byte offset
// in the round's 128 NS-byte piece space minus the lane offset, the chunk of pair P is real
// iff 256 P + 16 > t, i.e. P >= (t + 240) / 256.  An invalid or empty packet has t = 128 NS
// minus the lane offset: never real.
struct PairPlan {
  uint64_t db0, db1;
  int32_t p0, p1;  // first real pair of each DMA packet's chunk
};

struct RaggedRound {
  uint64_t cb;          // this lane's chunk address at slot 0
  int32_t top_slot;     // slot of this lane's top chunk (ns: packet has no whole word)
  uint32_t meta;        // round_meta(); the trailing-byte field holds z (bytes run past the end)
  uint32_t id;          // packet id (output index)
  // Wave-uniform, one SGPR each (the loop carries two rounds; every SGPR it carries is one the
  // job build and the round bodies cannot use, and the kernel is at the 106-SGPR limit):
  uint32_t hw;          // the round header's word (job build): ns | B << 26 | rot << 29 | line << 30 | fast << 31
  uint32_t d;           // the workgroup's round index (live, job number and job rounds follow from it)
  PairPlan plan;        // this lane's DMA plan for the round
  __device__ int32_t ns() const { return (int32_t)(hw & 0x3FFFFFFu); }  // slots of the round
  // B: the first top slot of a fast round (any of 0 .. 3 when ns == kPairMinSlots)
  __device__ int32_t top_uniform() const { return (int32_t)((hw >> 26) & 7u); }
  // top slots in B .. B + 1 (any in 4-slot rounds), no fallback, ns <= kRaggedFastMax
  __device__ bool fast() const { return (int32_t)hw < 0; }
  // a line round (line_round_from_record): whole-line slots, always fast
  __device__ bool line() const { return ((hw >> 30) & 1u) != 0u; }
  // a line round where some packet's a1 is not on the 16-B grid (r != 0: line_rotate, word masks)
  __device__ bool line_rot() const { return ((hw >> 29) & 1u) != 0u; }
};

constexpr int kRaggedFastMax = 14;  // unrolled round bodies for ns = kPairMinSlots .. kRaggedFastMax
constexpr int kLineMinSteps = 8;  // the shortest packets a line round holds (10: level, profiles/r06/line/)

// ---------------------------------------------------------------------------------
// Ragged rounds with 256-B loads.  The arithmetic and the compute
// slots are those of the rounds above (8 lanes x 8 packets, 128 B of each packet per compute
// slot); only the loads change.  A round runs an even number NS >= 4 of compute slots, and
// compute slots 2P, 2P + 1 of every packet -- one contiguous 256-B piece of it -- arrive
// together in "pair slot" P: two LDS-DMA instructions of 4 packets x 256 B each (instead of
// two instructions of 8 packets x 128 B, a slot apart): fewer packets and fewer partial
// lines per instruction.  Lane L of instruction i loads 16 B of packet 4 i + (L >> 4): half
// h = ((L >> 3) ^ (L >> 4)) & 1 of its piece (the halves of odd packets swapped, so that
// each compute slot's ds_read_b128 reads 256 distinct bytes per 16-lane quarter: no bank
// conflicts), chunk L & 7 of that half.  Compute lane 8 g + k then reads its chunk 7 - k of
// half 0 (compute slot 2P) and of half 1 (2P + 1) of packet g at fixed LDS offsets.
// Ring: 2 pair slots (4 KiB) per wave; consuming pair P, the DMAs of P + 1 and P + 2 are in
// flight.  The DMA lane decides per 16-B chunk whether it is real (at or after its packet's
// top word, not below the caller's buffer) or the zero chunk.
// ---------------------------------------------------------------------------------
constexpr int kPairRing = 2;                                    // pair slots per wave
// Lane k == 0 clears the z bytes past its packet's end in the last word (z in meta).
__device__ __forceinline__ uint32_t last_word_mask(uint32_t meta, uint32_t k) {
  // No lane compare (hipcc hoists k == 0 into a lane mask, then spills it to a VGPR lane):
  // kz = 0x18 on lane k == 0, else 0, by an arithmetic shift; the shift is 8 z there, else 0.
  const uint32_t kz = 0x18u & (uint32_t)((int32_t)(k - 1u) >> 31);
  return 0xFFFFFFFFu >> ((meta >> (kMetaNTailShift - 3)) & kz);
}

// Top-chunk masks from a 32-entry LDS table indexed by meta's head and v fields (5 bits):
// entry e = {m0..m3}, {x0..x3} with w_i <- (w_i & m_i) ^ x_i (mask_top's words, the initial
// register injected into the top word).  One asm statement: hipcc would put a plain LDS read
// behind the in-flight ring DMAs (vmcnt(0)).
struct TopMaskEntry {
  u32x4 m, x;
};
__device__ __forceinline__ void fill_top_masks(TopMaskEntry* t, uint32_t e) {
  if (e >= 32u) return;
  const uint32_t head = e & kMetaHeadMask, v = (e >> kMetaVShift) & 3u;
  uint32_t m[4] = {~0u, ~0u, ~0u, ~0u}, x[4] = {0u, 0u, 0u, 0u};
  if (head >= 1u && head <= 4u) {
    const uint32_t j0 = 4u - head;
    for (uint32_t i = 0; i < 4; ++i) {
      m[i] = i < j0 ? 0u : (i == j0 ? 0xFFFFFFFFu << (8u * v) : 0xFFFFFFFFu);
      x[i] = i == j0 ? head_k(v) : 0u;
    }
  } else if (head == kHeadZero) {  // line rounds: a chunk of the first line before the packet
    m[0] = m[1] = m[2] = m[3] = 0u;
  }
  t[e].m = u32x4{m[0], m[1], m[2], m[3]};
  t[e].x = u32x4{x[0], x[1], x[2], x[3]};
}
__device__ __forceinline__ void mask_top_lds(uint32_t meta, uint32_t table, uint32_t& w0, uint32_t& w1, uint32_t& w2,
                                             uint32_t& w3) {
  static_assert(kMetaHeadMask == 7 && kMetaVShift == 3, "the table index is meta & 0x1f");
  u32x4 m, x;
  uint32_t a;
  asm volatile(
      "v_bfe_u32 %2, %3, 0, 5\n\t"
      "v_lshl_add_u32 %2, %2, 5, %4\n\t"
      "ds_read_b128 %0, %2\n\t"
      "ds_read_b128 %1, %2 offset:16\n\t"
      "s_waitcnt lgkmcnt(0)"
      : "=&v"(m), "=&v"(x), "=&v"(a)
      : "v"(meta), "v"(table)
      : "memory");
  w0 = __builtin_amdgcn_bitop3_b32(w0, m.x, x.x, 0x6A);  // (w & m) ^ x
  w1 = __builtin_amdgcn_bitop3_b32(w1, m.y, x.y, 0x6A);
  w2 = __builtin_amdgcn_bitop3_b32(w2, m.z, x.z, 0x6A);
  w3 = __builtin_amdgcn_bitop3_b32(w3, m.w, x.w, 0x6A);
}
constexpr uint32_t kPairBytes = 2048;                           // one pair slot of one wave
constexpr uint32_t kPairStride = kWavesPerBlock * kPairBytes;   // bytes between ring positions
constexpr int kPairMinSlots = 4;                                // a round runs >= 2 pairs
static_assert(kPairMinSlots >= 2 * kPairRing, "a round's first kPairRing pairs come from the round before");


// From the two DMA packets' records (an invalid position reads as ax = info = 0: an empty
// packet, every chunk the zero chunk).  A packet whose top lies within 16 B of the caller's
// base also must not read below base4: its threshold is raised to that (o >= base4 - db).
__device__ __forceinline__ PairPlan pair_plan(uint64_t ax0, uint32_t info0, uint64_t ax1, uint32_t info1, int32_t ns,
                                              uint32_t dma_off, bool near_round, const LaneConsts& c) {
  // In pair units, so that no intermediate overflows (ns < 2^26 from u32 lengths):
  // (t + 240) / 256 = d / 2 + (128 (d & 1) + pad + 240 - lane offset) / 256, d = ns - nsteps.
  auto one = [&](uint64_t ax, uint32_t info, uint64_t& db) -> int32_t {
    const uint64_t piece0 = (ax & kRecAddrMask) - (uint64_t)kBytesPerStep * (uint64_t)ns;
    db = piece0 + dma_off;
    const uint32_t nsteps = info & kRecStepsMask, pad = (info >> kRecPadShift) << 2;
    const uint32_t d = (uint32_t)ns - nsteps;
    int32_t first = (int32_t)((d >> 1) + ((128u * (d & 1u) + pad + 240u - dma_off) >> 8));
    if (near_round && ((ax >> kRecNearBit) & 1u)) {  // o = 256 P + lane offset >= base4 - piece0
      const int64_t x = (int64_t)(c.base4 - piece0) - (int64_t)dma_off;
      const int64_t pb = x <= 0 ? 0 : (x + 255) >> 8;
      first = max(first, (int32_t)min(pb, (int64_t)0x40000000));
    }
    return first;
  };
  PairPlan p;
  p.p0 = one(ax0, info0, p.db0);
  p.p1 = one(ax1, info1, p.db1);
  return p;
}


// A pair round's per-lane state from its packet record and the round header (ns, B and
// `fast` are wave-uniform, from the job build's per-round max / min step counts).
__device__ __forceinline__ RaggedRound pair_round_from_record(uint64_t ax, uint32_t info, bool valid, uint32_t id,
                                                              const LaneConsts& c, uint32_t hw, bool near_round) {
  const uint64_t a1 = ax & kRecAddrMask;
  const int32_t nsteps = valid ? (int32_t)(info & kRecStepsMask) : 0;
  const uint32_t pad = (info >> kRecPadShift) << 2;
  const uint32_t v = (uint32_t)(ax >> kRecVShift) & 3u;
  const uint32_t z = (uint32_t)(ax >> kRecZShift) & 3u;
  RaggedRound rr;
  rr.hw = hw;
  const int32_t ns = rr.ns();
  // The top chunk's address, for the fallback load (near-base rounds only; unused otherwise).
  rr.cb = near_round ? a1 - 16u * (uint64_t)(c.k + 1u) - (uint64_t)kBytesPerStep * (uint64_t)(ns - 1) : 0ull;
  rr.top_slot = ns - nsteps;
  const int32_t rel = 112 - 16 * (int32_t)c.k - (int32_t)pad;
  const bool inside = nsteps > 0 && rel > -16;
  bool fb = false;
  if (near_round) {  // wave-uniform: only rounds holding a packet near the caller's base
    if (((ax >> kRecNearBit) & 1u) && valid && inside && rel < 0) {
      const uint64_t top = a1 - ((uint64_t)kBytesPerStep * (uint64_t)nsteps - pad);
      fb = top - c.base4 < (uint64_t)(-rel);
    }
  }
  const uint32_t head = inside && rel <= 0 ? (uint32_t)(rel / 4 + 4) : 0u;
  rr.meta = head | (v << kMetaVShift) | (nsteps == 0 ? kMetaEmpty : 0u) | (z << kMetaNTailShift) |
            (valid ? kMetaStore : 0u) | (fb ? kMetaFallback : 0u) | (inside && !fb ? kMetaDirect : 0u);
  rr.id = id;
  return rr;
}


// ---------------------------------------------------------------------------------
// Line rounds (round 6; host model: tests/test_line_rounds_model.py).  A round of 8 packets
// of one step count n in 8 .. 13 (no partial round, no packet near the caller's base) may run
// on whole 128-B lines instead of 128-B pieces ending at each packet's a1: compute slot s of
// packet g is the line NS - 1 - s lines before the packet's last line; a packet of n steps
// spans n or n + 1 lines, NS = the round's largest line count rounded up to even (the job build
// ORs a header bit for a packet of n + 1 lines), so every first line is slot B or B + 1.  Every DMA then reads whole lines, and the pairs that hold no line a
// neighbour shares (pairs 2 .. NS / 2 - 2) carry the non-temporal hint: tools/lines_probe,
// 1392-B packets 225.2 vs 254.5 us.  The arithmetic stays the 8-lane Horner on
// the 16-B grid ending at E16 = a1 rounded up to 16:
//   * lane k holds the chunks c = k mod 8 counted back from E16: chunk (j_last - k) mod 8 of
//     every line, j_last = the E16 chunk's index in the last line.  The DMA lane that fills
//     LDS position p (read by compute lane 7 - p) loads chunk (p + j_last + 1) mod 8;
//   * at the last slot the chunks past E16 (lanes k > j_last) and lane 0's words past a1 are
//     not multiplied in (the meta's skip mask): those streams keep their previous value;
//   * r = (E16 - a1) / 4: before the in-lane Horner, lane k forms the a1-grid chunk of its
//     class from its own words 0 .. 3 - r and lane (k + 1) mod 8's words 4 - r .. 3
//     (line_rotate; lane 7 takes lane 0's skipped words, one stream step behind);
//   * at its first line each lane masks its chunk from the mask table: before the first
//     word (kHeadZero), the first word's chunk (head, v: the init register injected), or none.
// ---------------------------------------------------------------------------------
// Packed round records (round 6; host model: tests/test_packed_records_model.py).  Once a
// job's round headers are complete, job_build writes the records of fast and line rounds in
// a form that already holds the round's slot count: what every lane of the round derives
// from it (its top slot and head code; each DMA lane's pair-0 address and first real pair)
// then costs a few instructions in make_round, instead of the full decode of the raw record
// per lane and round (8 lanes decode each packet, and each record is read by 3 lanes x its
// round; the build packs it once).  Generic and near-base rounds keep the raw record.
//   Fast rounds (format A, NS <= 14):
//     X = piece0 (48 bits: a1 - 128 NS) | W << 48,  W = 128 (NS - nsteps) + pad + 240 (12 bits)
//         -> db = piece0 + dma_off, first pair = (W - dma_off) >> 8 (pair_plan's formula)
//     Y = the meta of lane k_t (head h_t, v, empty, z, store) | k_t << 13 | top slot << 16 | id << 24
//         k_t = (127 - pad) >> 4 is the lane whose chunk holds the top word; the others' head is 0.
//   Line rounds (format B):
//     X = L (48 bits: the last line - 128 (NS - 1)) | j_last << 48 | x << 51 | m << 55,
//         x = NS - lines (the top slot), m = meta bits 3..9 (v, 0, z, r)
//     Y = head table (3 bits per lane k: kHeadZero, 4 - wt or 0) | id << 24
// Line and chunk indices use the addresses' low 32 bits (a packet spans < 2^25 lines).  GPU
// virtual addresses of packets are far above 1792 B, so piece0 and L never wrap below 0.
// ---------------------------------------------------------------------------------
constexpr int kPkWShift = 48;
constexpr uint32_t kPkKtShift = 13, kPkTopShift = 16, kPkIdShift = 24;
constexpr uint32_t kPkJlShift = 16, kPkXShift = 19, kPkMetaShift = 23;  // format B, in X's high word

// Format A from a raw record (valid: a packet is at this position; else ax = info = 0).
__device__ __forceinline__ void pack_fast(uint64_t ax, uint32_t info, bool valid, uint32_t ns, uint64_t& X,
                                          uint32_t& Y) {
  const uint64_t a1 = ax & kRecAddrMask;
  const uint32_t nsteps = valid ? info & kRecStepsMask : 0u, pad = valid ? (info >> kRecPadShift) << 2 : 0u;
  const uint32_t v = (uint32_t)(ax >> kRecVShift) & 3u, z = (uint32_t)(ax >> kRecZShift) & 3u;
  const uint32_t id = (uint32_t)(ax >> kJobLidShift) & 255u;
  const uint32_t W = 128u * (ns - nsteps) + pad + 240u;
  X = ((a1 - (uint64_t)kBytesPerStep * ns) & kRecAddrMask) | ((uint64_t)W << kPkWShift);
  const uint32_t kt = (127u - pad) >> 4;                    // rel = 112 - 16 k - pad in (-16, 0]
  const uint32_t ht = nsteps ? 32u - 4u * kt - (pad >> 2) : 0u;  // rel / 4 + 4
  Y = ht | (v << kMetaVShift) | (nsteps == 0 ? kMetaEmpty : 0u) | (z << kMetaNTailShift) |
      (valid ? kMetaStore : 0u) | (kt << kPkKtShift) | ((ns - nsteps) << kPkTopShift) | (id << kPkIdShift);
}

// Format B from a raw record of a line round (every position valid, NS = the round's slots).
__device__ __forceinline__ void pack_line(uint64_t ax, uint32_t info, uint32_t ns, uint64_t& X, uint32_t& Y) {
  const uint64_t a1 = ax & kRecAddrMask;
  const uint32_t a1l = (uint32_t)a1, nsteps = info & kRecStepsMask, pad = (info >> kRecPadShift) << 2;
  const uint32_t topl = a1l - (128u * nsteps - pad);
  const uint32_t lines = ((((a1l - 1u) >> 7) - (topl >> 7)) & 0x1FFFFFFu) + 1u;
  const uint32_t j_last = ((a1l - 1u) >> 4) & 7u, r = ((0u - a1l) >> 2) & 3u;
  const uint32_t jt = (topl >> 4) & 7u, ht = 4u - ((topl >> 2) & 3u);
  // Entry k is the code of chunk jk = (j_last - k) mod 8: kHeadZero for jk < jt, ht for jk = jt,
  // else 0.  Indexed by m = 7 - jk that is kHeadZero in the fields m >= 8 - jt and ht in field
  // 7 - jt; entry k is field (k + 7 - j_last) mod 8 of it, a rotation of the 24-bit word.
  // (The loop over k cost 45 VALU per packet; host model: tests/test_packed_records_model.py.)
  constexpr uint32_t kZeroRep = kHeadZero * 0x249249u;  // kHeadZero in all 8 fields
  const uint32_t rev = (kZeroRep & (0xFFFFFFu << (3u * (8u - jt)))) | (ht << (3u * (7u - jt)));
  const uint32_t rot = 3u * (7u - j_last);
  const uint32_t tab = ((rev >> rot) | (rev << (24u - rot))) & 0xFFFFFFu;
  const uint32_t v = (uint32_t)(ax >> kRecVShift) & 3u, z = (uint32_t)(ax >> kRecZShift) & 3u;
  const uint32_t m = v | (z << 3) | (r << 5);  // meta bits 3..9
  const uint64_t L = (((a1 - 1u) & ~127ull) - 128ull * (ns - 1u)) & kRecAddrMask;
  X = L | ((uint64_t)(j_last | ((ns - lines) << 3) | (m << 7)) << kPkWShift);
  Y = tab | (((uint32_t)(ax >> kJobLidShift) & 255u) << kPkIdShift);
}
static_assert(kPkJlShift == kPkWShift - 32 && kPkXShift == kPkJlShift + 3 && kPkMetaShift == kPkXShift + 4,
              "format B fields");

// A fast round's per-lane state from its format-A record.
__device__ __forceinline__ RaggedRound fast_round_decode(uint32_t Y, const LaneConsts& c, uint32_t hw) {
  RaggedRound rr;
  rr.hw = hw;
  rr.cb = 0;  // no fallback chunks in a fast round
  rr.top_slot = (int32_t)((Y >> kPkTopShift) & 15u);
  rr.meta = ((Y >> kPkKtShift) & 7u) == c.k ? Y : (Y & ~kMetaHeadMask);  // bits above 12: not meta fields
  rr.id = Y >> kPkIdShift;
  return rr;
}
__device__ __forceinline__ PairPlan fast_plan_decode(uint64_t X0, uint64_t X1, uint32_t dma_off) {
  auto one = [&](uint64_t X, uint64_t& db) -> int32_t {
    db = (X & kRecAddrMask) + dma_off;
    return (int32_t)(((uint32_t)(X >> 32) - (dma_off << 16)) >> 24);  // (W - dma_off) >> 8, W >= 240 >= dma_off
  };
  PairPlan pl;
  pl.p0 = one(X0, pl.db0);
  pl.p1 = one(X1, pl.db1);
  return pl;
}

// A line round's per-lane state from its format-B record: the head code of lane k from the
// table, the skip mask (lanes past E16 all 4 streams; lane 0 the words past a1).
__device__ __forceinline__ RaggedRound line_round_decode(uint64_t X, uint32_t Y, const LaneConsts& c, uint32_t hw) {
  const uint32_t xh = (uint32_t)(X >> 32);
  RaggedRound rr;
  rr.hw = hw;
  rr.cb = 0;  // no fallback chunks in a line round
  rr.top_slot = (int32_t)((xh >> kPkXShift) & 15u);
  const uint32_t j_last = (xh >> kPkJlShift) & 7u, r = (xh >> (kPkMetaShift + 5)) & 3u;
  const uint32_t head = (Y >> (3u * c.k)) & 7u;
  const uint32_t skip = (c.k > j_last ? 0xFu : 0u) | (c.k == 0u ? (0xF0u >> r) & 0xFu : 0u);
  rr.meta = head | ((xh >> (kPkMetaShift - 3)) & 0x3F8u) | kMetaStore | (skip << kMetaSkipShift);
  rr.id = Y >> kPkIdShift;
  return rr;
}
// The DMA plan of a line round: for each DMA packet, the lane's 16 B of pair 0 (half h of the
// pair: the line NS - 1 - h lines before the last one; chunk (p + j_last + 1) mod 8 of it) and
// the first pair whose line of half h is one of the packet's (earlier ones: the zero chunk).
__device__ __forceinline__ PairPlan line_plan_decode(uint64_t X0, uint64_t X1, uint32_t dma_off) {
  const uint32_t h128 = dma_off & 128u, p16 = (dma_off & 0x70u) + 16u;  // 128 h, 16 (p + 1)
  auto one = [&](uint64_t X, uint64_t& db) -> int32_t {
    const uint32_t xh = (uint32_t)(X >> 32);
    db = (X & kRecAddrMask) + (h128 | ((p16 + 16u * ((xh >> kPkJlShift) & 7u)) & 0x70u));
    const int32_t x = (int32_t)((xh >> kPkXShift) & 15u);
    return max(0, (x - (int32_t)(h128 >> 7) + 1) >> 1);
  };
  PairPlan pl;
  pl.p0 = one(X0, pl.db0);
  pl.p1 = one(X1, pl.db1);
  return pl;
}

// Before the in-lane Horner of a line round: the streams of this lane's a1-grid class,
// g_i = own word i - r for i >= r, else word i - r + 4 of lane (k + 1) mod 8 (ds_bpermute, in
// an asm statement with its own wait: hipcc would put a plain LDS access behind the ring DMAs).
__device__ __forceinline__ void line_rotate(uint32_t meta, uint32_t lane, uint32_t& h0, uint32_t& h1, uint32_t& h2,
                                            uint32_t& h3) {
  const uint32_t src = 4u * ((lane & ~7u) | ((lane + 1u) & 7u));
  uint32_t n1, n2, n3;
  asm volatile(
      "ds_bpermute_b32 %0, %3, %4\n\tds_bpermute_b32 %1, %3, %5\n\tds_bpermute_b32 %2, %3, %6\n\t"
      "s_waitcnt lgkmcnt(0)"
      : "=&v"(n1), "=&v"(n2), "=&v"(n3)
      : "v"(src), "v"(h1), "v"(h2), "v"(h3));
  // 4-way select by r as two bitop3 muxes per bit of r (0xD8: c ? b : a); as ternaries hipcc
  // made EXEC-masked branches of them.
  const uint32_t m0 = (uint32_t)((int32_t)(meta << (31 - kMetaLineRShift)) >> 31);      // r & 1
  const uint32_t m1 = (uint32_t)((int32_t)(meta << (31 - kMetaLineRShift - 1)) >> 31);  // r & 2
  auto pick = [&](uint32_t x0, uint32_t x1, uint32_t x2, uint32_t x3) {
    const uint32_t lo = __builtin_amdgcn_bitop3_b32(x0, x1, m0, 0xD8), hi = __builtin_amdgcn_bitop3_b32(x2, x3, m0, 0xD8);
    return __builtin_amdgcn_bitop3_b32(lo, hi, m1, 0xD8);
  };
  const uint32_t g0 = pick(h0, n3, n2, n1), g1 = pick(h1, h0, n3, n2), g2 = pick(h2, h1, h0, n3), g3 = pick(h3, h2, h1, h0);
  h0 = g0;
  h1 = g1;
  h2 = g2;
  h3 = g3;
}

// Per-lane constants of the pair ring.
struct PairRing {
  uint32_t topmask;  // LDS address of the top-chunk mask table (mask_top_lds)
  LdsVoid* slot0;    // this wave's pair slot 0
  uint32_t ring0;    // its LDS byte address
  uint32_t rd_a;     // this lane's read offset, half 0 (compute slot 2P)
  uint32_t dma_off;  // this lane's byte offset inside its DMA packets' 256-B pieces
  uint32_t q;        // pair slot of the pair being consumed (wave-uniform, 0 / 1)
  u32x4 nextv;       // landed data of the compute slot about to be consumed
  // Both DMAs of pair P of a round with plan pl into pair slot `slot`; `checked`: some chunk
  // of this pair may lie before its packet's top (or below the caller's buffer); `nt`: the
  // non-temporal hint (a line round's interior pairs; a compile-time constant where true).
  __device__ __forceinline__ void issue(const PairPlan& pl, int32_t P, uint32_t slot, bool checked,
                                        const LaneConsts& c, bool nt = false) {
    const uint64_t o = 256u * (uint64_t)P;
    uint64_t s0 = pl.db0 + o, s1 = pl.db1 + o;
    if (checked) {
      s0 = P >= pl.p0 ? s0 : c.dummy;
      s1 = P >= pl.p1 ? s1 : c.dummy;
    }
    LdsChar* const dst = (LdsChar*)slot0 + slot * kPairStride;
    if (nt) {
      __builtin_amdgcn_global_load_lds((const void*)s0, (LdsVoid*)dst, 16, 0, 2);
      __builtin_amdgcn_global_load_lds((const void*)s1, (LdsVoid*)(dst + 1024), 16, 0, 2);
    } else {
      __builtin_amdgcn_global_load_lds((const void*)s0, (LdsVoid*)dst, 16, 0, 0);
      __builtin_amdgcn_global_load_lds((const void*)s1, (LdsVoid*)(dst + 1024), 16, 0, 0);
    }
  }
  __device__ __forceinline__ uint32_t addr_a(uint32_t slot) const { return ring0 + slot * kPairStride + rd_a; }
  __device__ __forceinline__ uint32_t addr_b(uint32_t slot) const { return ring0 + slot * kPairStride + (rd_a ^ 128u); }
};

// Consume compute slot s of a round of ns slots (s even: half 0 of pair s / 2, in pair slot
// R.q): read the next compute slot's data into R.nextv (fused with the lookups of this slot
// when `look`) and, after a half-0 slot, refill the pair slot just emptied with pair
// s / 2 + 2 (of this round, or pair s / 2 + 2 - ns / 2 of the next).
// Waits: consuming pair P, the DMAs of P + 1 and P + 2 may be in flight (vmcnt(2)); DMAs
// complete in issue order.  kLine: a line round's own pairs 2 .. ns / 2 - 2 (whole lines no
// neighbour shares) carry the non-temporal hint.
template <bool kLook, bool kLine = false>
__device__ __forceinline__ void pair_step(int32_t s, int32_t ns, const PairPlan& cur, const PairPlan& nxt,
                                          PairRing& R, const LaneConsts& c, bool cur_checked, uint32_t& h0,
                                          uint32_t& h1, uint32_t& h2, uint32_t& h3, uint32_t w0, uint32_t w1,
                                          uint32_t w2, uint32_t w3) {
  const bool half0 = (s & 1) == 0;
  const uint32_t next_addr = half0 ? R.addr_b(R.q) : R.addr_a(R.q ^ 1u);
  constexpr int kWait = 2;  // the two DMAs of the pair after the one read may stay in flight
  if constexpr (kLook) {
    horner_step_and_read<kWait>(c.lk, h0, h1, h2, h3, w0, w1, w2, w3, next_addr, R.nextv);
  } else {
    R.nextv = read_landed_slot<kWait>(next_addr);
  }
  if (half0) {
    const int32_t f = s / 2 + kPairRing, np = ns / 2;  // the pair that refills pair slot R.q
    // Pairs 0 and 1 of a round may hold tops (fast rounds: slots B .. B + 1, B <= 1, or any of
    // a 4-slot round's): issued checked, whoever issues them.
    if (f < np)
      R.issue(cur, f, R.q, cur_checked || f < kPairMinSlots / 2, c, kLine && f >= 2 && f + 1 < np);
    else
      R.issue(nxt, f - np, R.q, true, c);
  } else {
    R.q ^= 1u;
  }
}

// A fast round (tops of every packet in compute slots T .. T + 1, or T .. 3 when NS = 4; no
// fallback): unrolled; the pairs it issues for itself (P >= 2) need no check.  kLine: a line
// round (line_round_from_record): at the last slot lane 0 masks the words past a1 and the
// skip mask keeps the streams whose last chunk (or word) lies past E16.
template <int NS, int T = 0, bool kLine = false>
__device__ __forceinline__ void pair_round_fast(const RaggedRound& cur, const PairPlan& pc, const PairPlan& pn,
                                                PairRing& R, const LaneConsts& c, uint32_t& h0, uint32_t& h1,
                                                uint32_t& h2, uint32_t& h3) {
  static_assert(NS % 2 == 0 && NS >= kPairMinSlots, "pair rounds");
  static_assert(T == 0 || T == 1 || NS == kPairMinSlots, "leading zero slots beyond 1 only in minimum rounds");
  constexpr int kMaskEnd = NS == kPairMinSlots ? kPairMinSlots - 1 : T + 1;  // last slot a top can be in
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    const u32x4 v = R.nextv;
    if (s < T) {
      pair_step<false, kLine>(s, NS, pc, pn, R, c, false, h0, h1, h2, h3, 0, 0, 0, 0);
      issue_order_fence();
      continue;
    }
    uint32_t w0 = v.x, w1 = v.y, w2 = v.z, w3 = v.w;
    if (s == NS - 1) {
      const uint32_t zm = last_word_mask(cur.meta, c.k);  // data only: before the injection in mask_top
      w3 &= zm;
      if (kLine && cur.line_rot()) {  // lane 0: the a1-grid's last word is word 3 - r of the E16 chunk
        const uint32_t r = (cur.meta >> kMetaLineRShift) & 3u;
        w2 &= r >= 1u ? zm : 0xFFFFFFFFu;
        w1 &= r >= 2u ? zm : 0xFFFFFFFFu;
        w0 &= r >= 3u ? zm : 0xFFFFFFFFu;
      }
    }
    if (s <= kMaskEnd) {
      const bool mine = cur.top_slot == s && (cur.meta & kMetaHeadMask);
      if (mine) mask_top_lds(cur.meta, R.topmask, w0, w1, w2, w3);  // EXEC-masked; skipped when no lane
    }
    if (s == T) {
      h0 = w0;  // first top slot: every stream is still zero (M32^32(0) = 0), no lookups
      h1 = w1;
      h2 = w2;
      h3 = w3;
      pair_step<false, kLine>(s, NS, pc, pn, R, c, false, h0, h1, h2, h3, 0, 0, 0, 0);
    } else if (kLine && s == NS - 1) {
      const uint32_t o0 = h0, o1 = h1, o2 = h2, o3 = h3;
      pair_step<true, kLine>(s, NS, pc, pn, R, c, false, h0, h1, h2, h3, w0, w1, w2, w3);
      // skip bit i set: stream i keeps o_i (bitop3 0xD8: sel ? o : h)
      auto keep = [&](int i) { return (uint32_t)((int32_t)(cur.meta << (31 - (int)kMetaSkipShift - i)) >> 31); };
      h0 = __builtin_amdgcn_bitop3_b32(h0, o0, keep(0), 0xD8);
      h1 = __builtin_amdgcn_bitop3_b32(h1, o1, keep(1), 0xD8);
      h2 = __builtin_amdgcn_bitop3_b32(h2, o2, keep(2), 0xD8);
      h3 = __builtin_amdgcn_bitop3_b32(h3, o3, keep(3), 0xD8);
    } else {
      pair_step<true, kLine>(s, NS, pc, pn, R, c, false, h0, h1, h2, h3, w0, w1, w2, w3);
    }
    issue_order_fence();
  }
}

template <int... T>
__device__ __forceinline__ bool pair_round_short(const RaggedRound& cur, const PairPlan& pc, const PairPlan& pn,
                                                 PairRing& R, const LaneConsts& c, uint32_t& h0, uint32_t& h1,
                                                 uint32_t& h2, uint32_t& h3, std::integer_sequence<int, T...>) {
  return ((cur.top_uniform() == T ? (pair_round_fast<kPairMinSlots, T>(cur, pc, pn, R, c, h0, h1, h2, h3), true)
                                : false) ||
          ...);
}

// Line rounds: NS = 8 .. 14 (step counts 8 .. 13), T = 0 or 1.
__device__ __forceinline__ bool line_round_dispatch(const RaggedRound& cur, const PairPlan& pc, const PairPlan& pn,
                                                    PairRing& R, const LaneConsts& c, uint32_t& h0, uint32_t& h1,
                                                    uint32_t& h2, uint32_t& h3) {
  const int32_t ns = cur.ns();
  if (cur.top_uniform() == 0) {
    if (ns == 8) return pair_round_fast<8, 0, true>(cur, pc, pn, R, c, h0, h1, h2, h3), true;
    if (ns == 10) return pair_round_fast<10, 0, true>(cur, pc, pn, R, c, h0, h1, h2, h3), true;
    if (ns == 12) return pair_round_fast<12, 0, true>(cur, pc, pn, R, c, h0, h1, h2, h3), true;
    if (ns == 14) return pair_round_fast<14, 0, true>(cur, pc, pn, R, c, h0, h1, h2, h3), true;
  } else {
    if (ns == 10) return pair_round_fast<10, 1, true>(cur, pc, pn, R, c, h0, h1, h2, h3), true;
    if (ns == 12) return pair_round_fast<12, 1, true>(cur, pc, pn, R, c, h0, h1, h2, h3), true;
    if (ns == 14) return pair_round_fast<14, 1, true>(cur, pc, pn, R, c, h0, h1, h2, h3), true;
  }
  return false;
}

// Fast rounds of NS = 6, 8, ..., kRaggedFastMax slots, T = 0 or 1.
template <int... I>
__device__ __forceinline__ bool pair_round_dispatch(const RaggedRound& cur, const PairPlan& pc, const PairPlan& pn,
                                                    PairRing& R, const LaneConsts& c, uint32_t& h0, uint32_t& h1,
                                                    uint32_t& h2, uint32_t& h3, std::integer_sequence<int, I...>) {
  if (cur.line()) return line_round_dispatch(cur, pc, pn, R, c, h0, h1, h2, h3);
  if (cur.ns() == kPairMinSlots)
    return pair_round_short(cur, pc, pn, R, c, h0, h1, h2, h3, std::make_integer_sequence<int, kPairMinSlots>{});
  if (cur.top_uniform() == 0)
    return ((cur.ns() == kPairMinSlots + 2 * (I + 1)
                 ? (pair_round_fast<kPairMinSlots + 2 * (I + 1), 0>(cur, pc, pn, R, c, h0, h1, h2, h3), true)
                 : false) ||
            ...);
  if (cur.top_uniform() == 1)
    return ((cur.ns() == kPairMinSlots + 2 * (I + 1)
                 ? (pair_round_fast<kPairMinSlots + 2 * (I + 1), 1>(cur, pc, pn, R, c, h0, h1, h2, h3), true)
                 : false) ||
            ...);
  return false;
}

// Any round: per-lane top slot and fallback chunks, runtime slot count, every pair checked.
__device__ __forceinline__ void pair_round_generic(const RaggedRound& cur, const PairPlan& pc, const PairPlan& pn,
                                                   PairRing& R, const LaneConsts& c, const uint32_t* lds,
                                                   uint32_t& h0, uint32_t& h1, uint32_t& h2, uint32_t& h3) {
  const int32_t ns = cur.ns();
  for (int32_t s = 0; s < ns; ++s) {
    const u32x4 v = R.nextv;
    uint32_t w0 = v.x, w1 = v.y, w2 = v.z, w3 = v.w;
    const bool top = s == cur.top_slot;
    if (__builtin_amdgcn_ballot_w64(top && (cur.meta & kMetaFallback))) {
      if (top && (cur.meta & kMetaFallback))
        load_top_words(cur.cb + (uint64_t)kBytesPerStep * (uint64_t)s, cur.meta, c.dummy, w0, w1, w2, w3);
    }
    if (s == ns - 1) w3 &= last_word_mask(cur.meta, c.k);
    if (__builtin_amdgcn_ballot_w64(top && (cur.meta & kMetaHeadMask))) {
      if (top && (cur.meta & kMetaHeadMask)) mask_top_lds(cur.meta, R.topmask, w0, w1, w2, w3);
    }
    h0 = horner_main(lds, h0, w0, c.lk);
    h1 = horner_main(lds, h1, w1, c.lk);
    h2 = horner_main(lds, h2, w2, c.lk);
    h3 = horner_main(lds, h3, w3, c.lk);
    pair_step<false>(s, ns, pc, pn, R, c, true, h0, h1, h2, h3, 0, 0, 0, 0);
    issue_order_fence();
  }
}

// ---------------------------------------------------------------------------------
// Ragged kernel with in-kernel job sort (the default ragged path; no pre-pass, no
// record scratch in HBM).  The batch is cut into jobs of up to kJobPackets consecutive
// packets; workgroup b takes jobs b, b + grid, b + 2 grid, ...  One wave builds a job
// into an LDS job slot: its descriptors arrive by LDS-DMA (phase A), and a round later
// the wave sorts the job's packets by step class (a counting sort over the 64 lanes,
// 4 packets per lane, DPP scans) and writes the job's round records into the slot
// (phase B).  All 16 waves then take the job's rounds from the workgroup's LDS round
// counter, exactly like the other DMA kernels (dynamic dispatch inside the workgroup),
// and leave each round's 8 checksums in the slot's result array; the wave that finishes
// a job's last round writes the job's checksums to HBM with one contiguous 16-B store per
// lane.  Jobs are built kJobAhead jobs ahead of the rounds being claimed; kJobSlots slots
// rotate.
//   * neighbouring packets (which share a 128-B line) are read by one CU within a few
//     rounds, so the shared line comes from L2 rather than twice from HBM;
//   * results leave as whole lines (the class-sorted order never reaches HBM);
//   * the records live in LDS only (round 2's region pre-pass wrote and re-read 16 B per packet
//     in HBM and cost one more launch).
// Every LDS access after the first DMA is an asm statement with its own wait (hipcc would
// order a plain LDS access behind the in-flight LDS-DMAs).  Same round bodies as
// round 2's region kernel (ragged_round_fast / _generic).
// ---------------------------------------------------------------------------------
constexpr int kJobPackets = 256;                                 // 4 per lane of the building wave
constexpr int kJobRounds = kJobPackets / kPacketsPerWave;        // 32
constexpr int kMinJobRounds = kJobRounds / 2;                   // launch_ragged: RJ = 16 .. 32 rounds per job
constexpr int kJobSlots = 4;                                     // job slots in LDS (the 64-KiB pair ring leaves room for 4)
constexpr int kJobAhead = 2;                                     // jobs built ahead of the one claimed
// The prologue builds every job the initial claims (rounds 0 .. 2 x 16 - 1) reach plus kJobAhead
// more, each into a slot of its own.
static_assert(kJobSlots >= (2 * kWavesPerBlock - 1) / kMinJobRounds + kJobAhead + 1, "prologue jobs need their slots");
static_assert(kBlock - 64 * kJobSlots >= 768, "fill_lds_from: the waves that do not build fill the tables");
constexpr uint32_t kJobRoundBytes = 96;                          // per round: u64 ax[8], u32 info[8]
constexpr uint32_t kJobRecBytes = kJobRounds * kJobRoundBytes;   // 3 KiB, also the descriptor staging
constexpr uint32_t kJobClassWords = 4;                           // 16 classes, 4 x 8 bits (no packet: not counted)
constexpr uint32_t kJobSpinLimit = 1u << 22;                     // give up rather than hang (never hit)
// Failure bits (g_fault_word, enet_crc_device_status): which wait gave up first in a wave.
constexpr uint32_t kFaultReady = 1u;     // a job's records never became ready
constexpr uint32_t kFaultConsumed = 2u;  // a job slot's previous job was never fully read
constexpr uint32_t kFaultFreed = 4u;     // a result slot's previous job was never flushed
static_assert(kJobPackets == 4 * 64, "4 packets per lane");
static_assert(kStepClasses == 4 * (int)kJobClassWords && kJobPackets <= 256, "job_build: 8-bit class fields, 4 per word");
static_assert(kJobRecBytes == kJobPackets * 12, "staging: u64 offsets + u32 lengths");

struct JobSlot {
  u32x4 rec[kJobRecBytes / 16];
  uint32_t res[kJobPackets];
  // Per round of the job, from the job build: the largest and the smallest step count of its
  // valid packets, and bit 0 = one of them begins within 16 B of the caller's base (a top
  // chunk may need the fallback).  The round's slot count and its body follow from these
  // alone (no cross-lane reduction per round).
  u32x4 hdr[kJobRounds];
};
struct RaggedJobsLds {
  uint32_t tables[kLdsDwords];
  u32x4 ring[kPairRing][kWavesPerBlock][kPairBytes / 16];
  JobSlot job[kJobSlots];
  uint32_t ready[kJobSlots];     // k + 1 once the workgroup's k-th job has its records here
  uint32_t consumed[kJobSlots];  // rounds of the slot's job whose records have been read
  uint32_t done[kJobSlots];      // rounds of the job whose checksums are in res
  uint32_t freed[kJobSlots];     // k + 1 once the k-th job's checksums are in HBM
  uint32_t next_dispatch;
  uint32_t failed;               // != 0 once a wave gave up a wait: later waits fail at once, nothing more is flushed
  TopMaskEntry topmask[32];      // mask_top_lds
  uint32_t res_dummy[64];        // publish(): where the lanes that hold no checksum store theirs
};
static_assert(sizeof(RaggedJobsLds) <= 160 * 1024, "LDS");
// LDS byte addresses of the jobs kernel's variables as constants: its one __shared__ object
// starts at LDS address 0 (checked at the kernel's start), so a member's address is its
// offset.  (Casting a member's generic address to the LDS space costs a null test per use,
// s_cmp_lg_u64 + s_cselect, and keeps the object's 64-bit generic address in two SGPRs.)
#define ENET_S_OFF(m) ((uint32_t)offsetof(RaggedJobsLds, m))
__device__ __forceinline__ uint32_t job_off(uint32_t slot) { return ENET_S_OFF(job) + slot * (uint32_t)sizeof(JobSlot); }

struct RaggedJobsBatch {
  uint64_t base;
  const uint64_t* offsets;
  const uint32_t* lengths;
  uint32_t count;        // < 2^32 (launch_ragged): the job arithmetic is 32-bit
  uint32_t njobs;
  uint32_t job_packets;  // packets per job (<= kJobPackets), chosen so every workgroup gets the same job count
  uint32_t* fault;       // this launch's failure word (device address; launch_ragged: FaultWord)
#ifdef ENET_CRC_TEST_HOOKS
  // Test build: workgroup 0 gives up the fault_kind wait (kFaultReady / kFaultConsumed /
  // kFaultFreed) of its (fault_k - 1)-th job (fault_k == 0: none).
  uint32_t fault_kind;
  uint32_t fault_k;
#endif
};

__device__ __forceinline__ uint32_t lds_ld32(uint32_t a) {
  uint32_t v;
  asm volatile("ds_read_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(a) : "memory");
  return v;
}
__device__ __forceinline__ u32x4 lds_ld128(uint32_t a) {
  u32x4 v;
  asm volatile("ds_read_b128 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(a) : "memory");
  return v;
}
__device__ __forceinline__ void lds_st32(uint32_t a, uint32_t v) {
  asm volatile("ds_write_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" : : "v"(a), "v"(v) : "memory");
}
__device__ __forceinline__ void lds_st32_nowait(uint32_t a, uint32_t v) {
  asm volatile("ds_write_b32 %0, %1" : : "v"(a), "v"(v) : "memory");
}
__device__ __forceinline__ uint32_t lds_add_rtn(uint32_t a, uint32_t v) {
  uint32_t old;
  asm volatile("ds_add_rtn_u32 %0, %1, %2\n\ts_waitcnt lgkmcnt(0)" : "=v"(old) : "v"(a), "v"(v) : "memory");
  return old;
}

// No-return add, not waited for (the next asm wait on lgkmcnt covers it).
__device__ __forceinline__ void lds_add_nowait(uint32_t a, uint32_t v) {
  asm volatile("ds_add_u32 %0, %1" : : "v"(a), "v"(v) : "memory");
}
__device__ __forceinline__ void lds_or_nowait(uint32_t a, uint32_t v) {
  asm volatile("ds_or_b32 %0, %1" : : "v"(a), "v"(v) : "memory");
}

// Spin (asleep) until the LDS word at `a` equals `want`.  kWaitOk, or kWaitGaveUp after
// kJobSpinLimit polls, or kWaitFailFast as soon as the workgroup's failed word (at `fail`)
// is set: one wave that gives up makes every later wait of its workgroup return at once,
// so a broken pipeline drains in one pass instead of one time-out per round.
enum : uint32_t { kWaitOk = 0, kWaitGaveUp = 1, kWaitFailFast = 2 };
__device__ __forceinline__ uint32_t lds_wait_eq(uint32_t a, uint32_t want, uint32_t fail) {
  for (uint32_t i = 0; i < kJobSpinLimit; ++i) {
    if (__builtin_amdgcn_readfirstlane(lds_ld32(a)) == want) return kWaitOk;
    if (__builtin_amdgcn_readfirstlane(lds_ld32(fail)) != 0u) return kWaitFailFast;
    __builtin_amdgcn_s_sleep(2);
  }
  return kWaitGaveUp;
}

// A wave gave up a wait: mark its workgroup failed (LDS) and write the failure bit into the
// launch's failure word in host memory (one vector store by lane 0, system scope, waited
// for; a racing writer can only replace one non-zero bit by another).
__device__ __forceinline__ void report_fault(uint32_t fail, uint32_t bit, uint32_t* w) {
  if ((threadIdx.x & 63u) != 0u) return;
  lds_st32(fail, bit);
  if (!w) return;
  asm volatile("global_store_dword %0, %1, off sc0 sc1\n\ts_waitcnt vmcnt(0)" : : "v"(w), "v"(bit) : "memory");
}

__global__ __launch_bounds__(kBlock) __attribute__((unused)) void crc32_ragged_jobs_kernel(RaggedJobsBatch b, uint32_t* __restrict__ out) {
  send_servers_home();
  // job_build's wait for its descriptor DMAs: every round issues one ring DMA per compute slot
  // (NS >= kPairMinSlots) after the job_dma of the iteration, so vmcnt(kDescWait) covers them.
  constexpr int kDescWait = 2;
  static_assert(kDescWait < kPairMinSlots, "a round issues >= kPairMinSlots DMAs after the descriptors'");
  __shared__ __attribute__((aligned(16))) RaggedJobsLds S;
  uint32_t* const lds = S.tables;
  constexpr uint32_t kLook = 2;  // a wave knows its current round and the next one
  const LaneConsts c = lane_consts(b.base);
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  // Wave w < kJobSlots clears job slot w's flags: the wave that builds into the slot in the
  // prologue clears them itself, in order before its build sets them.
  if (wv < (uint32_t)kJobSlots && lane == 0) {
    S.ready[wv] = 0;
    S.consumed[wv] = 0;
    S.done[wv] = 0;
    S.freed[wv] = 0;
  }
  if (threadIdx.x == kBlock - 1) {
    S.next_dispatch = kWavesPerBlock * kLook;
    S.failed = 0;
  }
  if ((uint32_t)(uintptr_t)(LdsVoid*)lds != 0) __builtin_trap();  // horner_step_and_read addresses

  auto job_of = [&](uint32_t k) -> uint32_t { return blockIdx.x + k * gridDim.x; };  // < njobs, or >= it past the end
  const uint32_t JP = b.job_packets;
  auto job_count = [&](uint32_t J) -> uint32_t {  // packets in job J (J < njobs)
    const uint64_t left = (uint64_t)b.count - (uint64_t)J * JP;
    return left < (uint64_t)JP ? (uint32_t)left : JP;
  };
  // Round d of this workgroup: round d % RJ of its (d / RJ)-th job, RJ = JP / 8 rounds
  // per job (only the batch's last job has fewer).  Monotone: once a round is past the
  // batch, so is every later one.
  const uint32_t RJ = JP / kPacketsPerWave;
  // d / RJ as one s_mul_hi: M = ceil(2^32 / RJ) is exact for d < 2^27 rounds (RJ <= 32;
  // launch_ragged keeps the rounds of a workgroup far below that).  hipcc's expansion of
  // the division is 11 scalar instructions, and this loop is issue-bound.
  const uint32_t rj_magic = 0xFFFFFFFFu / RJ + 1u;
  auto div_rj = [&](uint32_t x) -> uint32_t { return __umulhi(x, rj_magic); };
  auto round_valid = [&](uint32_t d) -> bool {
    const uint32_t k = div_rj(d);
    const uint32_t J = job_of(k);
    return J < b.njobs && (d - k * RJ) * kPacketsPerWave < job_count(J);
  };
  // This workgroup's jobs k = 0 .. wg_jobs - 1 (job J = blockIdx.x + k grid); only its last can
  // hold fewer than JP packets.  Per round then: live = d < wg_rounds, and the job's packet and
  // round counts by one scalar compare (no 64-bit job arithmetic per round).
  const uint32_t wg_jobs = (b.njobs - blockIdx.x + gridDim.x - 1) / gridDim.x;
  const uint32_t last_n = job_count(job_of(wg_jobs - 1u));
  const uint32_t last_rounds = (last_n + kPacketsPerWave - 1) / kPacketsPerWave;
  const uint32_t wg_rounds = (wg_jobs - 1u) * RJ + last_rounds;

  // Phase A: the descriptors of job J into the slot's record area (u64 offsets at +0,
  // u32 lengths at +2048): three 16-B DMAs per lane (kJobPackets descriptors from the
  // job's first; those past the job are never used), or, near the batch end, 4-B DMAs
  // clamped to the batch.
  auto job_dma = [&](uint64_t J, uint32_t slot) {
    LdsChar* st = (LdsChar*)&S.job[slot].rec[0];
    const uint64_t p0 = J * JP;
    if (p0 + kJobPackets <= b.count) {
      // The lane's byte offset through an asm statement: hipcc would otherwise hoist the three
      // per-lane addresses out of the round loop and spill them (a scratch reload, then
      // vmcnt(0), at every job build).
      uint32_t l16;
      asm volatile("v_lshlrev_b32 %0, 4, %1" : "=v"(l16) : "v"(lane));
      const char* const ob = reinterpret_cast<const char*>(b.offsets + p0) + l16;
      const char* const lb = reinterpret_cast<const char*>(b.lengths + p0) + l16;
      __builtin_amdgcn_global_load_lds((const void*)ob, (LdsVoid*)st, 16, 0, 0);
      __builtin_amdgcn_global_load_lds((const void*)(ob + 1024), (LdsVoid*)(st + 1024), 16, 0, 0);
      __builtin_amdgcn_global_load_lds((const void*)lb, (LdsVoid*)(st + 2048), 16, 0, 0);
    } else {
      // Not unrolled: one address live at a time (unrolled, hipcc hoisted all twelve out
      // of the round loop and spilled them to scratch: 18 MB of scratch writes per G2 launch).
      const uint32_t* offw = reinterpret_cast<const uint32_t*>(b.offsets);
#pragma unroll 1
      for (uint32_t i = 0; i < 12; ++i) {
        const uint32_t w = 64u * (i & 7u) + lane;
        const uint64_t e = i < 8 ? p0 + w / 2 : p0 + 64u * (i - 8u) + lane;
        const void* src = e >= b.count ? (const void*)g_zero_chunk
                          : i < 8    ? (const void*)(offw + 2 * e + (w & 1u))
                                     : (const void*)(b.lengths + e);
        __builtin_amdgcn_global_load_lds(src, (LdsVoid*)(st + 256 * i), 4, 0, 0);
      }
    }
  };
  // Phase B (>= kPairMinSlots ring DMAs after phase A): sort the job's packets by step class and
  // write its round records in place of the descriptors; then mark the slot ready.
  auto job_build = [&](uint64_t J, uint32_t slot, uint32_t gen) {
    asm volatile("s_waitcnt vmcnt(%0)" : : "i"(kDescWait) : "memory");
    const uint32_t st = (job_off(slot) + (uint32_t)offsetof(JobSlot, rec));
    u32x4 o01, o23, ln;
    asm volatile(  // one round trip
        "ds_read_b128 %0, %3\n\tds_read_b128 %1, %3 offset:16\n\tds_read_b128 %2, %4\n\ts_waitcnt lgkmcnt(0)"
        : "=&v"(o01), "=&v"(o23), "=&v"(ln)
        : "v"(st + 32u * lane), "v"(st + 2048u + 16u * lane)
        : "memory");
    const uint64_t off[4] = {o01.x | (uint64_t)o01.y << 32, o01.z | (uint64_t)o01.w << 32,
                             o23.x | (uint64_t)o23.y << 32, o23.z | (uint64_t)o23.w << 32};
    const uint32_t len[4] = {ln.x, ln.y, ln.z, ln.w};
    const uint32_t n = job_count(J);
    const uint32_t hdr = (job_off(slot) + (uint32_t)offsetof(JobSlot, hdr));
    if (lane < (uint32_t)kJobRounds) {  // max 0, min ~0, flags 0; in order before the atomics below
      asm volatile("ds_write_b128 %0, %1" : : "v"(hdr + 16u * lane), "v"(u32x4{0u, 0xFFFFFFFFu, 0u, 0u}) : "memory");
    }
    uint64_t ax[4];
    uint32_t info[4], cls[4], rank[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const bool v = 4u * lane + i < n;
      const RaggedRecord rec = ragged_record(b.base + off[i], len[i], c.base4);
      ax[i] = v ? rec.ax | ((uint64_t)(4u * lane + i) << kJobLidShift) : 0ull;
      info[i] = v ? rec.info : 0u;  // an invalid position reads as an empty packet at address 0 (pair_plan)
      cls[i] = v ? (rec.nsteps < kStepClasses - 1 ? rec.nsteps : kStepClasses - 1) : (uint32_t)kStepClasses;
      rank[i] = 0;
#pragma unroll
      for (int j = 0; j < i; ++j) rank[i] += cls[j] == cls[i] ? 1u : 0u;
    }
    // Class counts of this lane as 8-bit fields (class c: word c / 4, field c % 4; positions past
    // the job's packets are not counted, they keep their own index), their inclusive scan over the
    // lanes, the job's totals, and each class's first position, all in wrapping 32-bit words.  A
    // field reaches 256, or a sum of fields carries into the next field, only when every packet of
    // the job lies in that class or below: the carry lands in classes that hold no packet
    // (tests/test_job_sort_model.py restates this arithmetic and checks every position).
    uint32_t cnt[kJobClassWords];
#pragma unroll
    for (uint32_t w = 0; w < kJobClassWords; ++w) cnt[w] = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {  // bit 8 c of the 128-bit count word: one 64-bit shift, two selects
      const uint64_t one = 1ull << (8u * (cls[i] & 7u));
      const bool lo = cls[i] < 8u, hi = cls[i] - 8u < 8u;  // classes 0..7 / 8..15 (16: no packet)
      cnt[0] += lo ? (uint32_t)one : 0u;
      cnt[1] += lo ? (uint32_t)(one >> 32) : 0u;
      cnt[2] += hi ? (uint32_t)one : 0u;
      cnt[3] += hi ? (uint32_t)(one >> 32) : 0u;
    }
    uint32_t start[kJobClassWords];
    uint32_t run = 0;  // packets of the classes below word w (mod 256)
#pragma unroll
    for (uint32_t w = 0; w < kJobClassWords; ++w) {
      start[w] = wave_inclusive_add(cnt[w]);
      const uint32_t tot = (uint32_t)__builtin_amdgcn_readlane((int)start[w], 63);
      // field f: run + the totals of fields 0 .. f - 1 (tot x 0x01010100 sums the fields below)
      const uint32_t base = tot * 0x01010100u + (run & 255u) * 0x01010101u;
      run += (tot * 0x01010101u) >> 24;
      start[w] = start[w] - cnt[w] + base;
    }
    uint32_t qpos[4];  // each packet's position in the job's sorted order
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const uint32_t cw = cls[i] >> 2;
      const uint32_t sw = cw & 2u ? (cw & 1u ? start[3] : start[2]) : (cw & 1u ? start[1] : start[0]);
      const bool valid = cls[i] < (uint32_t)kStepClasses;
      const uint32_t q = valid ? ((sw >> (8u * (cls[i] & 3u))) & 255u) + rank[i] : 4u * lane + (uint32_t)i;
      qpos[i] = q;
      if (valid) {  // the round header
        const uint32_t h = hdr + 16u * (q >> 3), ns_i = info[i] & kRecStepsMask;
        asm volatile("ds_max_u32 %0, %1\n\tds_min_u32 %0, %1 offset:4" : : "v"(h), "v"(ns_i) : "memory");
        // bit 0: near the caller's base; bit 1: the packet spans nsteps + 1 lines (a line round
        // then needs one slot more); bit 2: its a1 is off the 16-B grid (line_rotate)
        const uint32_t a1l = (uint32_t)ax[i], topl = a1l - (128u * ns_i - ((info[i] >> kRecPadShift) << 2));
        const uint32_t flags = ((uint32_t)(ax[i] >> kRecNearBit) & 1u) |
                               (((((a1l - 1u) >> 7) - (topl >> 7)) & 0x1FFFFFFu) == ns_i ? 2u : 0u) |
                               (a1l & 12u ? 4u : 0u);
        if (flags) lds_or_nowait(h + 8u, flags);
      }
    }
    // Per round, make_round's rule evaluated once here: hdr.w = ns | B << 26 | fast << 31 (the
    // header's max / min / near are complete: this wave's LDS atomics above are processed
    // before its read below).
    if (lane < RJ) {
      const u32x4 hv = lds_ld128(hdr + 16u * lane);
      const int32_t mx = (int32_t)hv.x;
      const int32_t ns = max(kPairMinSlots, (mx + 1) & ~1), B = ns - mx;
      const bool two_pairs = ns <= kPairMinSlots;  // every pair of the round is issued checked
      const int32_t lim = two_pairs ? ns : B + 1;
      const bool partial = (lane + 1u) * kPacketsPerWave > n;
      const bool near = (hv.z & 1u) != 0u;
      // mx > 0: a round of empty packets only (B = 4) has no fast body (pair_round_short: B <= 3).
      const bool fast = !near && mx > 0 && ns <= kRaggedFastMax && (int64_t)ns - (int64_t)hv.y <= (int64_t)lim &&
                        (!partial || two_pairs);
      // A line round (format B, pack_line): 8 packets of one step count n in kLineMinSteps ..
      // 13, none near the caller's base.  They span n or n + 1 lines (n + 1 for some: header
      // bit 1); NS = that maximum rounded up to even, first lines in slots B .. B + 1.
      // Only when that costs no slot over the end-anchored round (an even n with a packet of
      // n + 1 lines would need two more: G2 +4 % with them, profiles/r06/line/).
      const int32_t ml = mx + (int32_t)((hv.z >> 1) & 1u), nl = (ml + 1) & ~1;
      const bool line = !near && !partial && hv.y == hv.x && mx >= kLineMinSteps && mx <= 13 && nl == ns;
      const uint32_t word = line ? (uint32_t)nl | ((uint32_t)(nl - ml) << 26) | ((hv.z & 4u) << 27) | 0xC0000000u
                                 : (uint32_t)ns | ((uint32_t)B << 26) | (fast ? 0x80000000u : 0u);
      lds_st32(hdr + 16u * lane + 12u, word);
    }
    // The records at their sorted positions: packed for fast and line rounds (this wave's
    // header words above are written before its reads below), raw for the others.
    uint32_t hwq[4];  // the header words of the packets' rounds, one round trip
    asm volatile(
        "ds_read_b32 %0, %4 offset:12\n\tds_read_b32 %1, %5 offset:12\n\t"
        "ds_read_b32 %2, %6 offset:12\n\tds_read_b32 %3, %7 offset:12\n\ts_waitcnt lgkmcnt(0)"
        : "=&v"(hwq[0]), "=&v"(hwq[1]), "=&v"(hwq[2]), "=&v"(hwq[3])
        : "v"(hdr + 16u * (qpos[0] >> 3)), "v"(hdr + 16u * (qpos[1] >> 3)), "v"(hdr + 16u * (qpos[2] >> 3)),
          "v"(hdr + 16u * (qpos[3] >> 3))
        : "memory");
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const uint32_t q = qpos[i], r = st + (q >> 3) * kJobRoundBytes, hw = hwq[i];
      uint64_t X = ax[i];
      uint32_t Y = info[i];
      if ((hw >> 30) & 1u)
        pack_line(ax[i], info[i], hw & 0x3FFFFFFu, X, Y);
      else if ((int32_t)hw < 0)
        pack_fast(ax[i], info[i], cls[i] < (uint32_t)kStepClasses, hw & 0x3FFFFFFu, X, Y);
      // not waited for: the ready flag below is written after them (LDS operations of a wave
      // complete in order), and its store waits
      asm volatile("ds_write_b64 %0, %1\n\tds_write_b32 %2, %3" : : "v"(r + 8u * (q & 7u)), "v"(X),
                   "v"(r + 64u + 4u * (q & 7u)), "v"(Y) : "memory");
    }
    if (lane == 0) lds_st32((ENET_S_OFF(ready) + 4u * slot), gen);
  };

  // Prologue (no ring DMA yet): wave w builds job w, for the jobs of the initial claims
  // (rounds 0 .. 2 x 16 - 1) and kJobAhead more; the claims of the loop (rounds >= 32)
  // build the rest.  RJ >= 16 (launch_ragged), so that is at most 2 + kJobAhead jobs.
  // The building waves fetch and sort their jobs while the other waves fill the tables (the
  // builds do not read the tables): the start is a descriptor fetch plus a build, not a table
  // fill, a barrier and then a build.
  const uint32_t first_jobs = (kWavesPerBlock * kLook - 1) / RJ + kJobAhead + 1;
  if (wv < first_jobs) {
    if (job_of(wv) < b.njobs) {
      job_dma(job_of(wv), wv);
      __builtin_amdgcn_s_waitcnt(0);
      job_build(job_of(wv), wv, wv + 1u);
    }
  } else {
    const uint32_t t0 = 64u * first_jobs;
    fill_lds_from(lds, threadIdx.x - t0, kBlock - t0);
    fill_top_masks(S.topmask, kBlock - 1u - threadIdx.x);
  }
  __syncthreads();

  // Jobs this wave has seen ready / flushed (a job's flags are polled once per wave).
  uint32_t seen_ready = 0, seen_freed = 0;
  const uint32_t fail_a = ENET_S_OFF(failed);
  // This lane's offset inside the 256-B pieces of its DMA packets (PairRing).
  const uint32_t dma_off = 128u * (((lane >> 3) ^ (lane >> 4)) & 1u) + 16u * (lane & 7u);
  // A wait's outcome: true if the flag came; a wave's own time-out is reported.
  auto waited = [&](uint32_t w, uint32_t bit) -> bool {
    if (w == kWaitGaveUp) report_fault(fail_a, bit, b.fault);
    return w == kWaitOk;
  };
  auto make_round = [&](uint32_t d) -> RaggedRound {
    uint64_t ax = 0;
    uint32_t info = 0;
    const uint32_t k = div_rj(d), slot = k % kJobSlots;
    bool rv = d < wg_rounds;  // round_valid(d)
    if (rv && k + 1u > seen_ready) {
      rv = waited(lds_wait_eq((ENET_S_OFF(ready) + 4u * slot), k + 1u, fail_a), kFaultReady);
      if (rv) seen_ready = k + 1u;
    }
#ifdef ENET_CRC_TEST_HOOKS
    if (rv && blockIdx.x == 0 && k + 1u == b.fault_k && b.fault_kind == kFaultReady) rv = waited(kWaitGaveUp, kFaultReady);
#endif
    u32x4 axd = {0, 0, 0, 0};  // the records of this lane's DMA packets lane / 16 and lane / 16 + 4
    uint64_t infod = 0;
    u32x4 hd = {0, 0, 0, 0};   // the round header: max steps, min steps, near flag
    if (rv) {
      const uint32_t r = (job_off(slot) + (uint32_t)offsetof(JobSlot, rec)) + (d - k * RJ) * kJobRoundBytes;
      const uint32_t gd = lane >> 4;
      asm volatile(  // one round trip
          "ds_read_b64 %0, %5\n\tds_read_b32 %1, %6\n\t"
          "ds_read2_b64 %2, %7 offset1:4\n\tds_read2_b32 %3, %8 offset1:4\n\t"
          "ds_read_b128 %4, %9\n\ts_waitcnt lgkmcnt(0)"
          : "=&v"(ax), "=&v"(info), "=&v"(axd), "=&v"(infod), "=&v"(hd)
          : "v"(r + 8u * c.grp), "v"(r + 64u + 4u * c.grp), "v"(r + 8u * gd), "v"(r + 64u + 4u * gd),
            "v"((job_off(slot) + (uint32_t)offsetof(JobSlot, hdr)) + 16u * (d - k * RJ))
          : "memory");
      if (lane == 0) lds_add_nowait((ENET_S_OFF(consumed) + 4u * slot), 1u);
    }
    // ns | B << 26 | fast << 31 (job build); a round without records: 4 slots, B = 0, not fast
    const uint32_t hw = rv ? __builtin_amdgcn_readfirstlane(hd.w) : (uint32_t)kPairMinSlots;
    const bool near_round = (__builtin_amdgcn_readfirstlane(hd.z) & 1u) != 0u;  // bit 1: line rounds' extra line
    const int32_t ns = (int32_t)(hw & 0x3FFFFFFu);
    const uint64_t ax0 = axd.x | (uint64_t)axd.y << 32, ax1 = axd.z | (uint64_t)axd.w << 32;
    // Rounds holding a packet near the caller's base (the batch's first few) take their own copy
    // of the decode: the others carry no near-base code at all (one scalar branch).
    RaggedRound rr;
    if ((hw >> 30) & 1u) {  // a line round (never near the base, never partial): format B
      rr = line_round_decode(ax, info, c, hw);
      rr.plan = line_plan_decode(ax0, ax1, dma_off);
    } else if ((int32_t)hw < 0) {  // a fast round (never near the base): format A
      rr = fast_round_decode(info, c, hw);
      rr.plan = fast_plan_decode(ax0, ax1, dma_off);
    } else if (near_round) {
      rr = pair_round_from_record(ax, info, rv && ((ax >> kRecValidBit) & 1u), (uint32_t)(ax >> kJobLidShift) & 255u,
                                  c, hw, true);
      rr.plan = pair_plan(ax0, (uint32_t)infod, ax1, (uint32_t)(infod >> 32), ns, dma_off, true, c);
    } else {
      rr = pair_round_from_record(ax, info, rv && ((ax >> kRecValidBit) & 1u), (uint32_t)(ax >> kJobLidShift) & 255u,
                                  c, hw, false);
      rr.plan = pair_plan(ax0, (uint32_t)infod, ax1, (uint32_t)(infod >> 32), ns, dma_off, false, c);
    }
    rr.d = d;
    return rr;
  };

  // A round's checksum (lane k == 0 of each group) into its job's result array; the last
  // round of a job writes the job's checksums to HBM.
  auto publish = [&](uint32_t k0, uint32_t id, uint32_t meta, uint32_t job_rounds, uint32_t reg) {
    // The round's checksums into the job's result array; the last round of a job
    // writes the job's checksums to HBM.
    const uint32_t slot0 = k0 % kJobSlots;
    if (k0 >= (uint32_t)kJobSlots && k0 + 1u - (uint32_t)kJobSlots > seen_freed) {
      if (waited(lds_wait_eq((ENET_S_OFF(freed) + 4u * slot0), k0 - (uint32_t)kJobSlots + 1u, fail_a), kFaultFreed))
        seen_freed = k0 + 1u - (uint32_t)kJobSlots;
    }
#ifdef ENET_CRC_TEST_HOOKS
    if (blockIdx.x == 0 && k0 >= (uint32_t)kJobSlots && k0 + 1u == b.fault_k && b.fault_kind == kFaultFreed)
      (void)waited(kWaitGaveUp, kFaultFreed);
#endif
    // The checksum store is not waited for on its own: the done counter's wait below covers
    // it (LDS operations complete in order).
    {  // every lane stores: lane k == 0 of a valid packet into res[id], the others into res_dummy
      const uint32_t sel = (uint32_t)((int32_t)(meta << (31 - 10)) >> 31) &  // kMetaStore (bit 10)
                           (uint32_t)((int32_t)(c.k - 1u) >> 31);            // k == 0
      const uint32_t ra = (job_off(slot0) + (uint32_t)offsetof(JobSlot, res)) + 4u * id, da = ENET_S_OFF(res_dummy) + 4u * lane;
      lds_st32_nowait((sel & ra) | (~sel & da), __builtin_bswap32(~reg));
    }
    uint32_t old = 0;
    if (lane == 0) old = lds_add_rtn((ENET_S_OFF(done) + 4u * slot0), 1u);
    old = __builtin_amdgcn_readfirstlane(old);
    // After a failure in the workgroup nothing more is flushed: a job whose records or
    // result slot were skipped would leave stale checksums in res[].
    if (old + 1u == job_rounds && __builtin_amdgcn_readfirstlane(lds_ld32(fail_a)) == 0u) {
      const uint64_t J0 = job_of(k0);
      const uint32_t n0 = job_count(J0);
      const u32x4 v = lds_ld128((job_off(slot0) + (uint32_t)offsetof(JobSlot, res)) + 16u * lane);
      // The lane's offset through an asm statement: hipcc would hoist the lane's output pointer
      // out of the round loop and spill it (a scratch reload per job).
      uint32_t l16;
      asm volatile("v_lshlrev_b32 %0, 4, %1" : "=v"(l16) : "v"(lane));
      uint32_t* dst = reinterpret_cast<uint32_t*>(reinterpret_cast<char*>(out + J0 * JP) + l16);
      if (4u * lane + 4u <= n0) {
        reinterpret_cast<U32x4A4*>(dst)->v = v;
      } else {
        if (4u * lane + 0u < n0) dst[0] = v.x;
        if (4u * lane + 1u < n0) dst[1] = v.y;
        if (4u * lane + 2u < n0) dst[2] = v.z;
      }
    }
    if (old + 1u == job_rounds) {
      if (lane == 0) {
        lds_st32((ENET_S_OFF(done) + 4u * slot0), 0u);
        lds_st32((ENET_S_OFF(freed) + 4u * slot0), k0 + 1u);
      }
    }
  };
  if (!round_valid(wv)) return;
  RaggedRound cur = make_round(wv);
  RaggedRound nxt = make_round(wv + kWavesPerBlock);
  PairRing R;
  R.slot0 = (LdsVoid*)&S.ring[0][wv][0];
  R.ring0 = (ENET_S_OFF(ring) + wv * kPairBytes);
  R.topmask = ENET_S_OFF(topmask);
  {
    const uint32_t g = lane >> 3, k = lane & 7u, j = g & 3u;
    R.rd_a = 1024u * (g >> 2) + 256u * j + 128u * (j & 1u) + 16u * (7u - k);
    R.dma_off = dma_off;
  }
  R.q = 0;
  R.issue(cur.plan, 0, 0, true, c);  // cur.ns >= kPairMinSlots: pairs 0 and 1
  R.issue(cur.plan, 1, 1, true, c);
  R.nextv = read_landed_slot<2>(R.addr_a(0));
  uint32_t tree_a = 0x10000u;  // tree_levels_asm's address register (high half 1, kept)
  while (cur.d < wg_rounds) {  // the current round is inside the batch
    uint32_t d = 0;
    if (lane == 0) d = lds_add_rtn(ENET_S_OFF(next_dispatch), 1u);
    d = __builtin_amdgcn_readfirstlane(d);
    // Build duty: the claimer of a job's first round builds the job kJobAhead later (the
    // prologue built the first ones) once every round of the slot's previous job has read
    // its record.  That wait never closes a cycle: a round's record is read at the end of
    // the iteration that claimed it, and nothing there waits for a younger job (the
    // checksum slot below waits only for an older job's flush).
    bool build = false;
    const uint32_t kd = div_rj(d), kb = kd + kJobAhead, bslot = kb % kJobSlots;
    if (d == kd * RJ && kb >= first_jobs && kb < wg_jobs) {  // rare: the first round of a job
      build = kb < (uint32_t)kJobSlots ||
              waited(lds_wait_eq((ENET_S_OFF(consumed) + 4u * bslot), RJ, fail_a), kFaultConsumed);
#ifdef ENET_CRC_TEST_HOOKS
      if (blockIdx.x == 0 && kb >= (uint32_t)kJobSlots && kb + 1u == b.fault_k && b.fault_kind == kFaultConsumed)
        build = waited(kWaitGaveUp, kFaultConsumed);
#endif
      if (build) {
        if (lane == 0) lds_st32((ENET_S_OFF(consumed) + 4u * bslot), 0u);
        job_dma(job_of(kb), bslot);
      }
    }
    uint32_t h0 = 0, h1 = 0, h2 = 0, h3 = 0;
    // Fast rounds (every valid packet's top in slots B .. B + 1, or anywhere in the shortest
    // rounds; no fallback chunk; NS <= kRaggedFastMax) take an unrolled body per NS, mixed-class
    // rounds included (round 4: 149.5 vs 157.8 us on G2); the others (fallback
    // chunks near the caller's base, longer or wider-spread rounds) the generic loop.
    // A fast round always has its body (its NS and B are those the header rule admits; the
    // record is packed for it, so the generic loop could not run it).
    if (cur.fast())
      (void)pair_round_dispatch(cur, cur.plan, nxt.plan, R, c, h0, h1, h2, h3,
                                std::make_integer_sequence<int, (kRaggedFastMax - kPairMinSlots) / 2>{});
    else
      pair_round_generic(cur, cur.plan, nxt.plan, R, c, lds, h0, h1, h2, h3);
    if (cur.line() && cur.line_rot()) line_rotate(cur.meta, lane, h0, h1, h2, h3);  // this lane's a1-grid streams
    uint32_t y = apply_rep(lds, h0, h1, c.lk.lp1, c.lk);  // in-lane Horner over the 4 word streams
    y = apply_rep(lds, y, h2, c.lk.lp1, c.lk);
    y = apply_rep(lds, y, h3, c.lk.lp1, c.lk);
    y = tree_levels_asm(y, tree_a);
    uint32_t reg = finish_word(lds, y, (cur.meta >> kMetaNTailShift) & 3u, c.lk);  // lane k == 0 holds it
    if (cur.meta & kMetaEmpty) reg = kInitRegister;
    {
      const uint32_t k0 = div_rj(cur.d);
      publish(k0, cur.id, cur.meta, k0 + 1u == wg_jobs ? last_rounds : RJ, reg);
    }
    if (build) job_build(job_of(kb), bslot, kb + 1u);
    const RaggedRound after = make_round(d);
    cur = nxt;
    nxt = after;
  }
  __builtin_amdgcn_s_waitcnt(0);
}


}  // namespace

int cu_count_for_current_device();

constexpr int kMaxRoundSteps = 14;  // NS 1..14 (packets up to 1792 B); NS >= 15 exceeds 128 VGPRs

template <bool kRagged>
struct Launcher {
  Batch<kRagged> b;
  uint32_t* out;
  hipStream_t stream;
  unsigned blocks;

  template <int NS>
  hipError_t rounds() {
    hipLaunchKernelGGL((crc32_rounds_kernel<NS, kRagged>), dim3(blocks), dim3(kBlock), 0, stream, b, out);
    return hipGetLastError();
  }
  hipError_t streaming() {
    hipLaunchKernelGGL((crc32_stream_kernel<kStreamDepth, kRagged>), dim3(blocks), dim3(kBlock), 0, stream, b,
                       out);
    return hipGetLastError();
  }
  template <int... I>
  hipError_t dispatch(int ns, std::integer_sequence<int, I...>) {
    hipError_t e = hipErrorInvalidValue;
    const bool hit = ((ns == I + 1 ? (e = rounds<I + 1>(), true) : false) || ...);
    return hit ? e : streaming();
  }
};

static unsigned grid_for(uint64_t count, hipError_t& err) {
  const int cus = cu_count_for_current_device();
  if (cus <= 0) {
    err = hipErrorNoDevice;
    return 0;
  }
  constexpr uint64_t kPacketsPerBlock = (uint64_t)kWavesPerBlock * kPacketsPerWave;
  uint64_t blocks = (count + kPacketsPerBlock - 1) / kPacketsPerBlock;
  if (blocks > (uint64_t)cus) blocks = (uint64_t)cus;
  err = hipSuccess;
  return (unsigned)blocks;
}

template <int NS>
static hipError_t launch_uniform_regs(const UniformBatch& u, uint32_t* out, hipStream_t stream, unsigned blocks) {
  hipLaunchKernelGGL((crc32_uniform_regs_kernel<NS>), dim3(blocks), dim3(kBlock), 0, stream, u, out);
  return hipGetLastError();
}

// Packets that all end on a 128-B line (e.g. 64 KiB buffers from an aligned base): the
// DMAs carry the non-temporal hint (every group slot is one whole line of its own).
static bool nt_lines(const UniformBatch& u) {
  const uint64_t lx = (u.length + 3u) & ~3u;
  return ((u.base + lx) & 127u) == 0 && (u.stride & 127u) == 0;
}

// ns in 1..kMaxRoundSteps only (the register ring holds a whole round).
template <int... I>
static hipError_t dispatch_uniform_regs(int ns, const UniformBatch& u, uint32_t* out, hipStream_t stream,
                                        unsigned blocks, std::integer_sequence<int, I...>) {
  hipError_t e = hipErrorInvalidValue;
  (void)((ns == I + 1 ? (e = launch_uniform_regs<I + 1>(u, out, stream, blocks), true) : false) || ...);
  return e;
}

// crc32_uniform_lines_kernel's batches: back to back, 16-B multiple lengths, from a 16-B
// aligned base.  `head` = the packets before the first one that starts on a 128-B line (0 for
// a line-aligned base; < 8, since L * h mod 128 runs through its residues within 128 /
// gcd(L, 128) <= 8 steps): they go through the register ring, the whole-line kernel starts
// at packet head.  False when no packet starts on a line (e.g. L = 1200 from base + 8).
static bool lines_shape(uint64_t base, uint64_t stride, uint32_t length, uint64_t& head) {
  if (stride != length || (length & 15u) != 0 || (base & 15u) != 0) return false;
  for (uint64_t h = 0; h < (uint64_t)kPacketsPerWave; ++h) {
    if (((base + h * length) & 127u) == 0) {
      head = h;
      return true;
    }
  }
  return false;
}

template <int NSL>
static hipError_t launch_uniform_lines(const UniformBatch& u0, uint32_t* out, hipStream_t stream, unsigned blocks) {
  UniformBatch u = u0;
  hipLaunchKernelGGL((crc32_uniform_lines_kernel<NSL>), dim3(blocks), dim3(kBlock), 0, stream, u, out);
  return hipGetLastError();
}

template <int... I>
static hipError_t dispatch_uniform_lines(int nsl, const UniformBatch& u, uint32_t* out, hipStream_t stream,
                                         unsigned blocks, std::integer_sequence<int, I...>) {
  hipError_t e = hipErrorInvalidValue;
  (void)((nsl == I + kUniformRing ? (e = launch_uniform_lines<I + kUniformRing>(u, out, stream, blocks), true)
                                  : false) ||
         ...);
  return e;
}

// Aligned uniform batches (base and stride multiples of 4): packets up to kMaxRoundSteps
// steps (<= 1792 B) run the register ring with line-split loads (the G1 path), packets of
// >= 4 KiB the wave-per-packet kernel, the lengths in between the 8-packets-per-wave
// LDS-DMA kernel.  Unaligned uniform batches: the round kernels of the register form.
hipError_t launch_uniform(const uint8_t* base, uint64_t stride, uint32_t length, uint64_t count,
                          uint32_t* out, hipStream_t stream) {
  if (count == 0) return hipSuccess;
  hipError_t err;
  const uint64_t b0 = (uint64_t)(uintptr_t)base;
  if (((b0 | stride) & 3u) == 0 && length > 0 && length <= 0xFFFFFFFCu) {
    // One launch covers the whole batch; packets run to the next 4-byte boundary.
    const int nsx = make_geo(0, (length + 3u) & ~3u).nsteps;
    const unsigned blocks = grid_for(count, err);
    if (err != hipSuccess) return err;
    const UniformBatch u{b0, stride, length, count};
    // Packets of >= 4 KiB: one wave per packet, 1-KiB contiguous loads; 64-KiB buffers
    // 338-346 us vs 371-374 us for the 8-packets-per-wave DMA kernel.
    if (length >= (uint32_t)kWaveRing * kWaveStep) {
      uint64_t wblocks = (count + kWavesPerBlock - 1) / kWavesPerBlock;
      const int cus = cu_count_for_current_device();
      if (wblocks > (uint64_t)cus) wblocks = (uint64_t)cus;
      if ((((length + 3u) & ~3u) + kWaveStep - 1) / kWaveStep % kWaveRegRing == 0) {
        if (nt_lines(u))
          hipLaunchKernelGGL((crc32_wave_regs_kernel<true>), dim3((unsigned)wblocks), dim3(kBlock), 0, stream, u, out);
        else
          hipLaunchKernelGGL((crc32_wave_regs_kernel<false>), dim3((unsigned)wblocks), dim3(kBlock), 0, stream, u, out);
        return hipGetLastError();
      }
      if (nt_lines(u))
        hipLaunchKernelGGL((crc32_wave_dma_kernel<true>), dim3((unsigned)wblocks), dim3(kBlock), 0, stream, u, out);
      else
        hipLaunchKernelGGL((crc32_wave_dma_kernel<false>), dim3((unsigned)wblocks), dim3(kBlock), 0, stream, u, out);
      return hipGetLastError();
    }
    if (nsx <= kMaxRoundSteps) {
      // Back-to-back 16-B-multiple packets from a 16-B aligned base: every line read once,
      // whole, non-temporal (crc32_uniform_lines_kernel) for the whole rounds from the first
      // packet on a line, the register ring for the < 8 packets before it and after the last
      // whole round.
      const int nsl = (int)((length + 127u) / 128u);
      uint64_t head = 0;
      const bool lines = lines_shape(b0, stride, length, head);
      const uint64_t whole = lines && count > head ? (count - head) / kPacketsPerWave * kPacketsPerWave : 0;
      if (lines && nsl >= kUniformRing && nsl <= kMaxRoundSteps && whole > 0) {
        const UniformBatch w{b0 + head * stride, stride, length, whole};
        const unsigned wblocks = grid_for(whole, err);
        if (err != hipSuccess) return err;
        err = dispatch_uniform_lines(nsl, w, out + head, stream, wblocks,
                                     std::make_integer_sequence<int, kMaxRoundSteps - kUniformRing + 1>{});
        const uint64_t rest = count - whole;  // the head and the tail: one launch
        if (err != hipSuccess || rest == 0) return err;
        UniformBatch t{b0, stride, length, rest};
        t.skip_at = head;
        t.skip = whole;
        const unsigned tblocks = grid_for(rest, err);
        if (err != hipSuccess) return err;
        return dispatch_uniform_regs(nsx, t, out, stream, tblocks, std::make_integer_sequence<int, kMaxRoundSteps>{});
      }
      return dispatch_uniform_regs(nsx, u, out, stream, blocks, std::make_integer_sequence<int, kMaxRoundSteps>{});
    }
    if (nt_lines(u))
      hipLaunchKernelGGL((crc32_uniform_dma_kernel<true>), dim3(blocks), dim3(kBlock), 0, stream, u, out);
    else
      hipLaunchKernelGGL((crc32_uniform_dma_kernel<false>), dim3(blocks), dim3(kBlock), 0, stream, u, out);
    return hipGetLastError();
  }
  const unsigned blocks = grid_for(count, err);
  if (err != hipSuccess) return err;
  // Packet starts cycle through phases (base + p*stride) mod 4: steps per packet.
  int hi = 0;
  for (uint64_t p = 0; p < 4 && p < count; ++p) {
    const int n = make_geo((b0 + p * stride) & 3u, length).nsteps;
    hi = n > hi ? n : hi;
  }
  Launcher<false> L{Batch<false>{b0, nullptr, nullptr, stride, length, count}, out, stream, blocks};
  if (hi >= 1 && hi <= kMaxRoundSteps) return L.dispatch(hi, std::make_integer_sequence<int, kMaxRoundSteps>{});
  return L.streaming();
}

hipError_t launch_single(const uint8_t* base, uint32_t length, uint32_t* out, hipStream_t stream) {
  Launcher<false> L{Batch<false>{(uint64_t)(uintptr_t)base, nullptr, nullptr, 0, length, 1}, out, stream, 1};
  return L.streaming();
}

// Below this many packets the sort costs more than the padding it saves.
constexpr uint64_t kSortMinPackets = 4096;

#ifdef ENET_CRC_TEST_HOOKS
// Test build only: the shape of the last jobs-kernel launch (enet_crc_debug_ragged_shape).
std::atomic<uint64_t> g_last_njobs{0}, g_last_job_packets{0}, g_last_grid{0};
#endif

hipError_t launch_ragged(const uint8_t* base, const uint64_t* offsets, const uint32_t* lengths,
                         uint64_t count, uint32_t* out, hipStream_t stream, uint32_t* fault) {
  if (count == 0) return hipSuccess;
  hipError_t err;
  const unsigned blocks = grid_for(count, err);
  if (err != hipSuccess) return err;
  Batch<true> b{(uint64_t)(uintptr_t)base, offsets, lengths, 0, 0, count};
  if (count > 0xFFFFFFFFull || count < kSortMinPackets) {
    Launcher<true> L{b, out, stream, blocks};
    return L.streaming();
  }
  // In-kernel job sort (crc32_ragged_jobs_kernel): one launch, no scratch.  Workgroups take jobs statically,
  // so the launch lasts as long as the busiest workgroup's ceil(njobs / grid) jobs: the job
  // size (16..32 rounds) is the one that minimises that makespan in rounds (1M packets on
  // 256 CUs: 32 rounds of 16 packets, 8 jobs each).
  constexpr uint64_t kRoundPackets = kPacketsPerWave, kMaxJobRounds = kJobRounds;
  const int cus = cu_count_for_current_device();
  if (cus <= 0) return hipErrorNoDevice;
  uint64_t jp = kMaxJobRounds * kRoundPackets, njobs = 0, best = ~0ull;
  for (uint64_t rj = kMaxJobRounds; rj >= kMinJobRounds; --rj) {
    const uint64_t p = rj * kRoundPackets, nj = (count + p - 1) / p;
    const uint64_t grid = nj < (uint64_t)cus ? nj : (uint64_t)cus;
    const uint64_t span = (nj + grid - 1) / grid * rj;
    if (span < best) {
      best = span;
      jp = p;
      njobs = nj;
    }
  }
  const unsigned jblocks = (unsigned)(njobs < (uint64_t)cus ? njobs : (uint64_t)cus);
  // The kernel divides a workgroup's round index by RJ with one s_mul_hi, exact below 2^27
  // rounds (div_rj); a batch whose busiest workgroup would go past that (a device with few
  // CUs and billions of packets) takes the streaming kernel instead.
  const uint64_t wg_rounds = (njobs + jblocks - 1) / jblocks * (jp / kRoundPackets) + 2 * kWavesPerBlock;
  if (wg_rounds >= (1ull << 27)) {
    Launcher<true> L{b, out, stream, blocks};
    return L.streaming();
  }
  // Without a word of its own the launch reports into the device's (asynchronous entries).
  if (!fault) {
    int dev = 0;
    FaultWord w;
    if ((err = hipGetDevice(&dev)) != hipSuccess || (err = device_fault_word(dev, &w)) != hipSuccess) return err;
    fault = w.dev;
  }
  RaggedJobsBatch jb{b.base, offsets, lengths, (uint32_t)count, (uint32_t)njobs, (uint32_t)jp, fault};
#ifdef ENET_CRC_TEST_HOOKS
  // Test build only (tests/test_gpu_hooks.py): ENET_CRC_TEST_JOB_FAULT=<kind>:<k> makes
  // workgroup 0 give up its <kind> wait (ready, consumed, freed) for its (k-1)-th job; a
  // bare number means ready.
  jb.fault_kind = 0;
  jb.fault_k = 0;
  if (const char* fk = getenv("ENET_CRC_TEST_JOB_FAULT")) {
    const char* colon = strchr(fk, ':');
    jb.fault_kind = kFaultReady;
    if (colon) {
      const size_t n = (size_t)(colon - fk);
      jb.fault_kind = (n == 8 && !strncmp(fk, "consumed", 8)) ? kFaultConsumed
                      : (n == 5 && !strncmp(fk, "freed", 5)) ? kFaultFreed
                                                             : kFaultReady;
      fk = colon + 1;
    }
    jb.fault_k = (uint32_t)atoi(fk);
  }
  g_last_njobs = njobs;
  g_last_job_packets = jp;
  g_last_grid = jblocks;
#endif
  hipLaunchKernelGGL(crc32_ragged_jobs_kernel, dim3(jblocks), dim3(kBlock), 0, stream, jb, out);
  return hipGetLastError();
}

}  // namespace enet_crc

#ifdef ENET_CRC_TEST_HOOKS
// Test build only: {jobs, packets per job, workgroups} of the last ragged jobs launch.
extern "C" __attribute__((visibility("default"))) void enet_crc_debug_ragged_shape(uint64_t* out) {
  out[0] = enet_crc::g_last_njobs;
  out[1] = enet_crc::g_last_job_packets;
  out[2] = enet_crc::g_last_grid;
}
#endif
