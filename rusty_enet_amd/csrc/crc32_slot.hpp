// Checksum-slot arithmetic for batched ENet receive-verify and send-insert
// (SURVEY.md §8(b) "semantics that must survive batching", §8(f)1-2).
//
// Reference: the receive path overwrites the 4-byte checksum slot of a datagram
// with peer.connect_id (or 0 for peer id 4095) before checksumming it
// (src/c/protocol.rs:1470-1502); the send path writes connect_id (or 0) into the slot,
// checksums header+slot+commands and writes the checksum into the slot
// (src/c/protocol.rs:2255-2293).  The slot value is known only when the datagram is
// processed, so a batch is checksummed with whatever the slot holds and corrected
// afterwards, using the linearity of the CRC register over GF(2):
//
//   reg(m) = M8^L(0xFFFFFFFF) ^ A(m),  A linear,  checksum = bswap32(~reg).
//   Changing the slot's little-endian u32 by dv (XOR) changes A by
//   M8^n(M32(dv)), n = bytes after the slot: before the slot the zero-initialised
//   register stays 0, the 4 slot bytes give M32(dv), the n trailing zero bytes M8^n.
//   So  checksum(slot = v) = checksum(slot = u) ^ bswap32(M8^n(M32(u ^ v))).
//
// M8^n = M8^(n & 3) o M32^(n >> 2); M32^q is applied bit by bit of q through a
// ladder of operator tables L[k] = M32^(2^k), k < kSlotLevels = 32 (n is a u32).  L[0] table 3 is the reference CRC table (src/crc32.rs:1-34).
#pragma once
#include <stdint.h>

#include "crc32_geometry.hpp"  // ENET_HD
#include "crc32_ops.hpp"

namespace enet_crc {

constexpr int kSlotLevels = 32;
constexpr uint32_t kSlotLevelDwords = 4 * 256;

// ladder[k * 1024 + t * 256 + b] = M32^(2^k)(b << 8t).  Built on the host (the
// constexpr kOpTables holds the first kOpLevels levels; the rest by squaring).
inline void build_slot_ladder(uint32_t* ladder) {
  const OpTables& T = kOpTables;
  for (int k = 0; k < kOpLevels; ++k)
    for (int t = 0; t < 4; ++t)
      for (int b = 0; b < 256; ++b) ladder[k * 1024 + t * 256 + b] = T.op[k][t][b];
  for (int k = kOpLevels; k < kSlotLevels; ++k) {
    const uint32_t* prev = ladder + (k - 1) * 1024;
    auto apply_prev = [&](uint32_t x) {
      return prev[x & 0xffu] ^ prev[256 + ((x >> 8) & 0xffu)] ^ prev[512 + ((x >> 16) & 0xffu)] ^ prev[768 + (x >> 24)];
    };
    for (int t = 0; t < 4; ++t)
      for (uint32_t b = 0; b < 256; ++b) ladder[k * 1024 + t * 256 + b] = apply_prev(apply_prev(b << (8 * t)));
  }
}

// Inverse levels (after the kSlotLevels forward levels of the same device buffer):
// inv[k * 1024 + t * 256 + b] = M32^-(2^k)(b << 8t), k < kInvLevels, which undo up to
// 4 * (2^kInvLevels - 1) zero bytes (the flat ragged kernel's step-end alignment: <= 128).
// M8^-1(y) = ((y ^ T[b]) << 8) | b with b = inv_top[y >> 24] (crc32_ops.hpp).
constexpr int kInvLevels = 6;
constexpr int kLadderLevels = kSlotLevels + kInvLevels;

inline void build_inverse_ladder(uint32_t* inv) {
  const OpTables& T = kOpTables;
  auto m8inv = [&](uint32_t y) {
    const uint32_t b = T.inv_top[y >> 24];
    return ((y ^ T.sarwate[b]) << 8) | b;
  };
  for (int t = 0; t < 4; ++t)
    for (uint32_t b = 0; b < 256; ++b) {
      uint32_t x = b << (8 * t);
      for (int i = 0; i < 4; ++i) x = m8inv(x);
      inv[t * 256 + b] = x;
    }
  for (int k = 1; k < kInvLevels; ++k) {
    const uint32_t* prev = inv + (k - 1) * 1024;
    auto apply_prev = [&](uint32_t x) {
      return prev[x & 0xffu] ^ prev[256 + ((x >> 8) & 0xffu)] ^ prev[512 + ((x >> 16) & 0xffu)] ^ prev[768 + (x >> 24)];
    };
    for (int t = 0; t < 4; ++t)
      for (uint32_t b = 0; b < 256; ++b) inv[k * 1024 + t * 256 + b] = apply_prev(apply_prev(b << (8 * t)));
  }
}

// After the inverse levels: init[len] = M8^len(0xFFFFFFFF) for len < kInitTabLen (the
// initial register's share of a len-byte packet's register; flat ragged kernels).
constexpr uint32_t kInitTabLen = 1u << 16;
constexpr size_t kLadderDwords = (size_t)kLadderLevels * kSlotLevelDwords + kInitTabLen;

inline void build_init_table(uint32_t* t) {
  uint32_t v = kInitRegister;
  for (uint32_t n = 0; n < kInitTabLen; ++n) {
    t[n] = v;
    v = (v >> 8) ^ kOpTables.sarwate[v & 0xffu];
  }
}

ENET_HD uint32_t ladder_apply(const uint32_t* level, uint32_t x) {
  return level[x & 0xffu] ^ level[256 + ((x >> 8) & 0xffu)] ^ level[512 + ((x >> 16) & 0xffu)] ^ level[768 + (x >> 24)];
}

// bswap32(M8^n(M32(dv))): the change of the checksum when the slot's u32 changes by dv
// and n bytes follow the slot.  Levels k < fast_levels are read from `fast` (the LDS
// copy in the fix-up kernel), higher ones from `full` (all kSlotLevels levels).
ENET_HD uint32_t slot_delta(const uint32_t* fast, int fast_levels, const uint32_t* full, uint32_t dv, uint32_t n) {
  uint32_t r = ladder_apply(fast, dv);     // M32(dv): level 0
  const uint32_t* crc_table = fast + 768;  // M32(b << 24) == M8(b): the CRC table
  for (uint32_t i = 0; i < (n & 3u); ++i) r = (r >> 8) ^ crc_table[r & 0xffu];
  uint32_t q = n >> 2;
  for (int k = 0; q != 0; ++k, q >>= 1) {
    if (q & 1u) r = ladder_apply((k < fast_levels ? fast : full) + k * kSlotLevelDwords, r);
  }
  return __builtin_bswap32(r);
}

// Ladder levels slot_delta reads for n trailing bytes (always >= 1: level 0 is M32).
ENET_HD int slot_levels_for(uint32_t n) {
  const uint32_t q = n >> 2;
  int k = 1;
  while (k < 32 && (q >> k)) ++k;
  return k;
}

}  // namespace enet_crc
