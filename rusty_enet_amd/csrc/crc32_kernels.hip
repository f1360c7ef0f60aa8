// CDNA4 (gfx950) kernels for the ENet per-datagram CRC-32.
//
// Reference: jabuwu/rusty_enet src/crc32.rs:39-47 (one serial Sarwate chain per
// call).  Here every packet of a batch is checksummed by a GROUP of G lanes of a
// wavefront; a wave holds 64/G packets at once.
//
// Per packet (DESIGN.md §3 has the derivation):
//   * The packet's bytes [s, e) are viewed as little-endian 32-bit words on the
//     4-byte grid that ends at a1 = e & ~3.  Word d (d = 1 is the last) lives at
//     a1 - 4d.  The zero-initialised register after the words is
//         R = XOR_d M32^d (w_d),  M32 = "advance over 32 zero bits".
//   * Chunk c (16 bytes, words d = 4c+4 .. 4c+1) belongs to lane k = c mod G.
//     Each of the lane's four word slots is an independent Horner stream with
//     step W = 4G words:  h <- M32^W(h) ^ w.  One replicated LDS operator table
//     (M32^W) serves every step; the first (top) step needs no lookup.
//   * Bytes before s in the top word are masked off and the 0xFFFFFFFF initial
//     register is injected by XOR-ing head_k[s & 3] into that word.
//   * Combine: in-lane Horner with M32 over the four slots, then a log2(G)
//     level DPP/shuffle tree with fixed shifts M32^(4*2^l), then one M32.  All
//     shifts are fixed, so no variable-distance GF(2) multiply is ever needed.
//   * Trailing e & 3 bytes: Sarwate steps (src/crc32.rs:43) on lane 0.
//   * Output: bswap32(~R)  ==  (!crc).to_be()  (src/crc32.rs:46).
//
// LDS (one 1024-thread workgroup per CU, 144 KiB):
//   [0, 128 KiB)  M32^W tables, replicated 32x so that lane l always reads bank
//                 l%32 (conflict-free ds_read_b32).  Table k, entry i, bank b at
//                 dword (k>>1)*16384 + i*64 + (k&1)*32 + b.  The byte address is
//                 built with ONE v_perm_b32: byte1 = register byte k, byte0 =
//                 lane*4, byte2 = table pair.
//   [128 KiB, +) unreplicated small operators: M32^1 (set 0) and the tree
//                 operators M32^(4*2^(l-1)) (set l).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "crc32_ops.hpp"
#include "crc32_kernels.hpp"

namespace enet_crc {

__device__ const OpTables g_op_tables = kOpTables;

namespace {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
// 16 bytes at a 4-byte-aligned address (global_load_dwordx4; gfx950 runs in
// unaligned-access mode).
struct __attribute__((packed, aligned(4))) U32x4A4 {
  u32x4 v;
};

constexpr int kBlock = 1024;
constexpr int kWavesPerBlock = kBlock / 64;
constexpr uint32_t kMainDwords = 32768;  // 4 tables x 256 entries x 32 banks

constexpr int ilog2(int x) { return x <= 1 ? 0 : 1 + ilog2(x >> 1); }

template <int G>
struct Layout {
  static_assert(G == 2 || G == 4 || G == 8 || G == 16, "lanes per packet");
  static constexpr int kStreams = 4 * G;         // words per group step
  static constexpr int kMainLevel = ilog2(kStreams);
  static constexpr int kTreeLevels = ilog2(G);
  static constexpr int kSmallSets = 1 + kTreeLevels;
  static constexpr uint32_t kLdsDwords = kMainDwords + kSmallSets * 1024;
  static_assert(kMainLevel < kOpLevels, "operator table level");
};

// Global-address-space loads from integer addresses (keeps them global_load_*,
// not flat_*: flat loads also count on lgkmcnt and would serialise with the
// LDS table lookups).
typedef __attribute__((address_space(1))) const uint32_t GlobalU32;
typedef __attribute__((address_space(1))) const U32x4A4 GlobalU32x4A4;

__device__ __forceinline__ uint32_t load_word(uintptr_t addr) {
  return *reinterpret_cast<GlobalU32*>(addr);
}

__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}

__device__ __forceinline__ uint32_t lds_at(const uint32_t* lds, uint32_t byte_addr) {
  return *reinterpret_cast<const uint32_t*>(reinterpret_cast<const char*>(lds) + byte_addr);
}

// h' = M32^W(h) ^ w through the replicated tables.  lp0 = lane*4, lp1 = lane*4 | 64 KiB.
__device__ __forceinline__ uint32_t horner_main(const uint32_t* lds, uint32_t h, uint32_t w,
                                                uint32_t lp0, uint32_t lp1) {
  const uint32_t a0 = __builtin_amdgcn_perm(h, lp0, 0x0C020400u);
  const uint32_t a1 = __builtin_amdgcn_perm(h, lp0, 0x0C020500u);
  const uint32_t a2 = __builtin_amdgcn_perm(h, lp1, 0x0C020600u);
  const uint32_t a3 = __builtin_amdgcn_perm(h, lp1, 0x0C020700u);
  const uint32_t t0 = lds_at(lds, a0);
  const uint32_t t1 = lds_at(lds, a1 + 128u);
  const uint32_t t2 = lds_at(lds, a2);
  const uint32_t t3 = lds_at(lds, a3 + 128u);
  return xor3(xor3(t0, t1, t2), t3, w);
}

// M32^n(x) through an unreplicated 4x256 table set.
__device__ __forceinline__ uint32_t apply_small(const uint32_t* set, uint32_t x) {
  return xor3(set[x & 0xffu], set[256 + ((x >> 8) & 0xffu)], set[512 + ((x >> 16) & 0xffu)]) ^
         set[768 + (x >> 24)];
}

__device__ __forceinline__ uint32_t head_k(uint32_t v) {
  return v == 0 ? kOpTables.head_k[0]
                : (v == 1 ? kOpTables.head_k[1] : (v == 2 ? kOpTables.head_k[2] : kOpTables.head_k[3]));
}

template <int G>
__device__ __forceinline__ void fill_lds(uint32_t* lds) {
  using L = Layout<G>;
  const int t = threadIdx.x;  // (table k, entry i) pairs: 4 x 256 = kBlock
  {
    const int k = t >> 8, i = t & 255;
    const uint32_t v = g_op_tables.op[L::kMainLevel][k][i];
    const u32x4 vv = {v, v, v, v};
    u32x4* dst = reinterpret_cast<u32x4*>(lds + (k >> 1) * 16384 + i * 64 + (k & 1) * 32);
#pragma unroll
    for (int j = 0; j < 8; ++j) dst[j] = vv;
  }
  for (int x = t; x < L::kSmallSets * 1024; x += kBlock) {
    const int set = x >> 10, rem = x & 1023;
    const int level = set == 0 ? 0 : set + 1;
    lds[kMainDwords + x] = g_op_tables.op[level][rem >> 8][rem & 255];
  }
}

template <int G>
__device__ __forceinline__ u32x4 load_chunk(uintptr_t a1, uint32_t k, int64_t i) {
  const uintptr_t addr = a1 - 16u * (uintptr_t)(k + (uint64_t)G * (uint64_t)i + 1u);
  return reinterpret_cast<GlobalU32x4A4*>(addr)->v;
}

// CRC register (before finalisation) of bytes [sa, ea) for the group's lane k.
// Valid on lane k == 0 only.
template <int G>
__device__ __forceinline__ uint32_t group_crc_register(const uint32_t* lds, uintptr_t sa, uintptr_t ea,
                                                       uint32_t k, uint32_t lp0, uint32_t lp1) {
  using L = Layout<G>;
  const uintptr_t top = sa & ~(uintptr_t)3;
  const uintptr_t a1 = ea & ~(uintptr_t)3;
  const uint64_t nwords = (uint64_t)(a1 - top) >> 2;
  uint32_t reg = kInitRegister;
  if (nwords > 0) {
    const uint64_t nchunks = (nwords + 3) >> 2;
    const int64_t nsteps = (int64_t)((nchunks + G - 1) / G);
    uint32_t h0, h1, h2, h3;
    {  // top step: may start before sa; per-word loads with masking
      const int64_t c = (int64_t)k + (int64_t)G * (nsteps - 1);
      const int64_t rel0 = (int64_t)(a1 - top) - 16 * (c + 1);
      uint32_t w[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int64_t rel = rel0 + 4 * j;
        uint32_t x = 0;
        if (rel >= 0) x = load_word(top + (uintptr_t)rel);
        if (rel == 0) {
          const uint32_t v = (uint32_t)(sa - top);
          x = (x & (0xFFFFFFFFu << (8 * v))) ^ head_k(v);
        }
        w[j] = x;
      }
      h0 = w[0]; h1 = w[1]; h2 = w[2]; h3 = w[3];
    }
    // Remaining steps: whole 16-byte chunks, three loads in flight per lane.
    int64_t i = nsteps - 2;
    u32x4 q0 = {0, 0, 0, 0}, q1 = {0, 0, 0, 0}, q2 = {0, 0, 0, 0};
    if (i >= 0) q0 = load_chunk<G>(a1, k, i);
    if (i >= 1) q1 = load_chunk<G>(a1, k, i - 1);
    if (i >= 2) q2 = load_chunk<G>(a1, k, i - 2);
    while (i >= 0) {
      h0 = horner_main(lds, h0, q0.x, lp0, lp1);
      h1 = horner_main(lds, h1, q0.y, lp0, lp1);
      h2 = horner_main(lds, h2, q0.z, lp0, lp1);
      h3 = horner_main(lds, h3, q0.w, lp0, lp1);
      if (i >= 3) q0 = load_chunk<G>(a1, k, i - 3);
      if (--i < 0) break;
      h0 = horner_main(lds, h0, q1.x, lp0, lp1);
      h1 = horner_main(lds, h1, q1.y, lp0, lp1);
      h2 = horner_main(lds, h2, q1.z, lp0, lp1);
      h3 = horner_main(lds, h3, q1.w, lp0, lp1);
      if (i >= 3) q1 = load_chunk<G>(a1, k, i - 3);
      if (--i < 0) break;
      h0 = horner_main(lds, h0, q2.x, lp0, lp1);
      h1 = horner_main(lds, h1, q2.y, lp0, lp1);
      h2 = horner_main(lds, h2, q2.z, lp0, lp1);
      h3 = horner_main(lds, h3, q2.w, lp0, lp1);
      if (i >= 3) q2 = load_chunk<G>(a1, k, i - 3);
      --i;
    }
    // Combine the 4G streams.
    const uint32_t* m1 = lds + kMainDwords;
    uint32_t y = apply_small(m1, h0) ^ h1;
    y = apply_small(m1, y) ^ h2;
    y = apply_small(m1, y) ^ h3;
#pragma unroll
    for (int l = 1; l <= L::kTreeLevels; ++l) {
      const uint32_t t = apply_small(lds + kMainDwords + l * 1024, y);
      y ^= (uint32_t)__shfl_down((int)t, 1 << (l - 1), G);
    }
    reg = apply_small(m1, y);
  }
  return reg;
}

// Sarwate steps over the trailing (< 4) bytes [max(a1, sa), ea): src/crc32.rs:43.
__device__ __forceinline__ uint32_t tail_bytes(const uint32_t* sarwate, uint32_t reg, uintptr_t sa,
                                               uintptr_t ea) {
  const uintptr_t a1 = ea & ~(uintptr_t)3;
  const uintptr_t ts = a1 > sa ? a1 : sa;
  if (ts < ea) {
    const uint32_t w = load_word(a1);
    for (uintptr_t b = ts; b < ea; ++b) {
      const uint32_t byte = (w >> (8u * (uint32_t)(b - a1))) & 0xffu;
      reg = (reg >> 8) ^ sarwate[(reg ^ byte) & 0xffu];
    }
  }
  return reg;
}

template <int G, bool kRagged>
__global__ __launch_bounds__(kBlock) void crc32_packets_kernel(const uint8_t* __restrict__ base,
                                                              const uint64_t* __restrict__ offsets,
                                                              const uint32_t* __restrict__ lengths,
                                                              uint64_t stride, uint32_t length,
                                                              uint64_t count, uint32_t* __restrict__ out) {
  using L = Layout<G>;
  __shared__ __attribute__((aligned(16))) uint32_t lds[L::kLdsDwords];
  fill_lds<G>(lds);
  __syncthreads();

  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t k = lane & (G - 1);
  const uint32_t lp0 = (lane & 31u) << 2;
  const uint32_t lp1 = lp0 | 0x10000u;
  const uint32_t* sarwate = lds + kMainDwords + 768;  // op[0] table 3 == CRC table
  constexpr uint64_t kGroupsPerWave = 64 / G;
  const uint64_t wave = (uint64_t)blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6);
  const uint64_t total_groups = (uint64_t)gridDim.x * kWavesPerBlock * kGroupsPerWave;

  for (uint64_t p = wave * kGroupsPerWave + lane / G; p < count; p += total_groups) {
    uint64_t s, len;
    if constexpr (kRagged) {
      s = offsets[p];
      len = lengths[p];
    } else {
      s = p * stride;
      len = length;
    }
    const uintptr_t sa = (uintptr_t)base + s;
    const uintptr_t ea = sa + len;
    uint32_t reg = group_crc_register<G>(lds, sa, ea, k, lp0, lp1);
    if (k == 0) {
      reg = tail_bytes(sarwate, reg, sa, ea);
      out[p] = __builtin_bswap32(~reg);
    }
  }
}

}  // namespace

int cu_count_for_current_device();

template <int G, bool kRagged>
static hipError_t launch_packets(const uint8_t* base, const uint64_t* offsets, const uint32_t* lengths,
                                 uint64_t stride, uint32_t length, uint64_t count, uint32_t* out,
                                 hipStream_t stream) {
  if (count == 0) return hipSuccess;
  const int cus = cu_count_for_current_device();
  if (cus <= 0) return hipErrorNoDevice;
  constexpr uint64_t kGroupsPerBlock = (uint64_t)kWavesPerBlock * (64 / G);
  uint64_t blocks = (count + kGroupsPerBlock - 1) / kGroupsPerBlock;
  if (blocks > (uint64_t)cus) blocks = (uint64_t)cus;
  hipLaunchKernelGGL((crc32_packets_kernel<G, kRagged>), dim3((unsigned)blocks), dim3(kBlock), 0, stream,
                     base, offsets, lengths, stride, length, count, out);
  return hipGetLastError();
}

hipError_t launch_uniform(const uint8_t* base, uint64_t stride, uint32_t length, uint64_t count,
                          uint32_t* out, hipStream_t stream) {
  return launch_packets<8, false>(base, nullptr, nullptr, stride, length, count, out, stream);
}

hipError_t launch_ragged(const uint8_t* base, const uint64_t* offsets, const uint32_t* lengths,
                         uint64_t count, uint32_t* out, hipStream_t stream) {
  return launch_packets<8, true>(base, offsets, lengths, 0, 0, count, out, stream);
}

}  // namespace enet_crc
