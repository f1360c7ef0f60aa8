// Packet -> chunk geometry shared by the gfx950 kernel and its host-side model
// (tests/cpp/kernel_sim.cpp).  Pure integer arithmetic, __host__ __device__.
//
// A packet's bytes [sa, ea) are covered by little-endian 32-bit words on the
// 4-byte grid ending at a1 = ea & ~3 (the < 4 trailing bytes [a1, ea) are
// finished with byte steps).  The grid's first word is the one holding sa:
// top = sa & ~3.  16-byte chunk c (c = 0 is the LAST chunk) is [a1-16(c+1),
// a1-16c); it belongs to lane k = c % kLanesPerPacket at step i = c / kLanesPerPacket.
// Steps run from nsteps-1 (the top, possibly partial, chunk) down to 0.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#define ENET_HD __host__ __device__ __forceinline__
#else
#define ENET_HD inline
#endif

namespace enet_crc {

constexpr int kLanesPerPacket = 8;                  // G: lanes cooperating on one packet
constexpr int kPacketsPerWave = 64 / kLanesPerPacket;
constexpr int kBytesPerStep = 16 * kLanesPerPacket;  // one dwordx4 per lane per step

struct PacketGeo {
  uint64_t sa, ea, top, a1;
  int32_t nsteps;  // 0 when the packet holds no whole grid word (then only byte steps)
};

ENET_HD PacketGeo make_geo(uint64_t sa, uint64_t len) {
  PacketGeo g;
  g.sa = sa;
  g.ea = sa + len;
  g.top = sa & ~(uint64_t)3;
  g.a1 = g.ea & ~(uint64_t)3;
  const uint64_t nwords = (g.a1 - g.top) >> 2;  // a1 >= top because ea >= sa
  g.nsteps = (int32_t)((((nwords + 3) >> 2) + kLanesPerPacket - 1) / kLanesPerPacket);
  return g;
}

// Signed byte offset of lane k's chunk at step i relative to `ref`:
//   (a1 - 16*(k + G*i + 1)) - ref.
ENET_HD int64_t chunk_offset(const PacketGeo& g, uint32_t k, int32_t i, uint64_t ref) {
  return (int64_t)(g.a1 - ref) - 16 * ((int64_t)k + (int64_t)kLanesPerPacket * i + 1);
}

// Kinds of load a (lane, step) issues.
enum ChunkKind : int {
  kChunkNone = 0,      // chunk entirely before the packet (or step beyond the packet): read zeros
  kChunkDirect = 1,    // 16 bytes at the chunk address (all inside [base4, a1))
  kChunkFallback = 2,  // chunk starts before the caller's buffer: per-word loads, rare
};

// base4 = caller's base pointer rounded down to 4: nothing below it is ever read.
ENET_HD int chunk_kind(const PacketGeo& g, uint32_t k, int32_t i, uint64_t base4) {
  if (i < 0 || i >= g.nsteps) return kChunkNone;
  if (chunk_offset(g, k, i, g.top) <= -16) return kChunkNone;
  if (chunk_offset(g, k, i, base4) < 0) return kChunkFallback;
  return kChunkDirect;
}

// Lane geometry of crc32_uniform_lines_kernel (back-to-back packets of L = 16 n bytes from a
// 128-B aligned base; group g of a round reads the round's lines [g L / 128, (g+1) L / 128)),
// shared with its host model (tests/cpp/kernel_sim.cpp).  nsl = ceil(L / 128) slots per round.
struct LinesLane {
  int64_t off0;     // byte offset of this lane's slot-0 chunk from its round's start
  bool dummy0;      // slot 0 reads the zero chunk (the group has NSL - 1 lines)
  uint32_t am[2];   // slot s in {0, 1}: AND mask of the data words (0: chunk of packet g - 1)
  uint32_t xm[2];   // slot s in {0, 1}: XOR into word 0 (the initial register)
  bool keep[2];     // slot s in {0, 1}: keep the raw chunk for group g - 1
  bool lo;          // takes a step-0 chunk from group g + 1
  uint32_t src4;    // ds_bpermute byte address of that chunk's lane
};

ENET_HD LinesLane lines_lane(uint32_t L, int nsl, uint32_t g, uint32_t k) {
  LinesLane r;
  const uint32_t lg = g * L / 128u, lg1 = (g + 1u) * L / 128u;
  const int first = nsl - (int)(lg1 - lg);  // 0 or 1
  const uint32_t jg = (g * L % 128u) / 16u, j1 = ((g + 1u) * L % 128u) / 16u, j2 = ((g + 2u) * L % 128u) / 16u;
  const uint32_t m = (j1 + 7u - k) & 7u;  // (j1 - 1 - k) mod 8
  r.off0 = 128 * ((int64_t)lg1 - nsl) + 16 * (int64_t)m;
  r.dummy0 = first == 1;
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    r.am[s] = first == s && m < jg ? 0u : 0xFFFFFFFFu;
    r.xm[s] = first == s && m == jg ? 0xFFFFFFFFu : 0u;
    r.keep[s] = first == s;
  }
  r.lo = k < j1;
  r.src4 = 4u * (g < 7u ? 8u * (g + 1u) + ((j2 + 8u - j1 + k) & 7u) : 8u * g + k);
  return r;
}

}  // namespace enet_crc
