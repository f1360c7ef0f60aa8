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

}  // namespace enet_crc
