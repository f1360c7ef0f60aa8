// Host-only pieces of the C ABI (no HIP): the host operator ladder, the byte-balanced
// shard split, the checksum merge and slot correction, and the staging-chunk plan of
// the host-memory path.  enet_crc_abi.hip uses them; tests/cpp/host_asan.cpp builds them
// with g++ -fsanitize=address,undefined next to the C oracle (make asan).
#pragma once
#include <stddef.h>
#include <stdint.h>

#include <algorithm>

#include "crc32_ops.hpp"
#include "crc32_slot.hpp"

namespace enet_crc {

// The ladder of crc32_slot.hpp (forward levels, inverse levels, init table), built once.
inline const uint32_t* host_slot_ladder() {
  static uint32_t* ladder = [] {
    uint32_t* l = new uint32_t[kLadderDwords];
    build_slot_ladder(l);
    build_inverse_ladder(l + kSlotLevels * kSlotLevelDwords);
    build_init_table(l + kLadderLevels * kSlotLevelDwords);
    return l;
  }();
  return ladder;
}

// Byte-balanced contiguous split (the same cut points as rusty_enet_amd/shards.py
// shard_bounds): cut k is one past the first packet whose cumulative byte end reaches
// floor(total * k / n).  lengths == NULL: an even split of `count` packets.
inline void split_bounds(const uint32_t* lengths, uint64_t count, uint32_t n, uint64_t* b) {
  b[0] = 0;
  b[n] = count;
  if (!lengths) {
    for (uint32_t k = 1; k < n; ++k) b[k] = (uint64_t)((unsigned __int128)count * k / n);
    return;
  }
  unsigned __int128 total = 0;
  for (uint64_t i = 0; i < count; ++i) total += lengths[i];
  uint64_t i = 0;
  unsigned __int128 end = count ? lengths[0] : 0;  // byte end of packet i
  for (uint32_t k = 1; k < n; ++k) {
    const unsigned __int128 target = total * k / n;
    if (target == 0 || count == 0) {
      b[k] = 0;
      continue;
    }
    while (end < target && i + 1 < count) end += lengths[++i];
    b[k] = i + 1;
  }
}

// The slot rule of crc32_slot.hpp as a host function: the checksum of a datagram
// whose 4-byte slot (followed by n bytes) holds new_slot instead of old_slot.
inline uint32_t slot_adjust_checksum(uint32_t crc, uint32_t old_slot, uint32_t new_slot, uint32_t n) {
  const uint32_t* l = host_slot_ladder();
  return crc ^ slot_delta(l, kSlotLevels, l, old_slot ^ new_slot, n);
}

// reg(a || b) = M8^n(reg(a) ^ 0xFFFFFFFF) ^ reg(b) with n = |b| (the initial register's
// share of reg(b) is M8^n(0xFFFFFFFF)), and reg = ~bswap32(checksum), so
//   checksum(a || b) = bswap32(M8^n(bswap32(crc_a))) ^ crc_b.
// M8^n = M8^(n mod 4) M32^(n / 4): byte steps, then the host ladder's M32^(2^k) tables
// (4 lookups per set bit) while n / 4 < 2^32; beyond that by binary powering of M8 as a
// 32 x 32 GF(2) matrix (column i = M8(1 << i)).
inline uint32_t combine_checksums(uint32_t crc_a, uint32_t crc_b, uint64_t len_b) {
  if (len_b == 0) return crc_a;
  if ((len_b >> 2) < (1ull << kSlotLevels)) {
    const uint32_t* l = host_slot_ladder();
    uint32_t r = __builtin_bswap32(crc_a);
    for (uint64_t i = 0; i < (len_b & 3u); ++i) r = (r >> 8) ^ kOpTables.sarwate[r & 0xffu];
    uint64_t q = len_b >> 2;
    for (int k = 0; q != 0; ++k, q >>= 1)
      if (q & 1u) r = ladder_apply(l + (size_t)k * kSlotLevelDwords, r);
    return __builtin_bswap32(r) ^ crc_b;
  }
  auto apply = [](const uint32_t* m, uint32_t x) {
    uint32_t r = 0;
    for (int i = 0; x != 0; ++i, x >>= 1)
      if (x & 1u) r ^= m[i];
    return r;
  };
  uint32_t op[32], sq[32];
  for (int i = 0; i < 32; ++i) {
    const uint32_t x = 1u << i;
    op[i] = (x >> 8) ^ kOpTables.sarwate[x & 0xffu];  // M8, src/crc32.rs:43 with a zero byte
  }
  uint32_t v = __builtin_bswap32(crc_a);
  for (uint64_t n = len_b;;) {
    if (n & 1u) v = apply(op, v);
    n >>= 1;
    if (n == 0) break;
    for (int i = 0; i < 32; ++i) sq[i] = apply(op, op[i]);
    for (int i = 0; i < 32; ++i) op[i] = sq[i];
  }
  return __builtin_bswap32(v) ^ crc_b;
}

// One staging chunk of the host-memory path: packets [first, end) whose byte span
// [lo, hi) fits `max_bytes` (a single longer packet makes a chunk of its own) and at most
// `max_packets` packets.  lo_al = lo rounded down to 4: the device copy keeps the host
// bytes' offset mod 4, so the kernels see the same word grid.  span = hi - lo_al.
struct StageChunk {
  uint64_t end, lo_al, span;
};

inline StageChunk plan_stage_chunk(const uint64_t* offsets, const uint32_t* lengths, uint64_t count, uint64_t first,
                                   uint64_t max_bytes, uint64_t max_packets) {
  uint64_t lo = offsets[first], hi = offsets[first] + lengths[first];
  uint64_t q = first + 1;
  while (q < count && q - first < max_packets) {
    const uint64_t nlo = std::min<uint64_t>(lo, offsets[q]);
    const uint64_t nhi = std::max<uint64_t>(hi, offsets[q] + lengths[q]);
    if (nhi - nlo > max_bytes) break;
    lo = nlo;
    hi = nhi;
    ++q;
  }
  const uint64_t lo_al = lo & ~(uint64_t)3;
  return StageChunk{q, lo_al, hi - lo_al};
}

}  // namespace enet_crc
