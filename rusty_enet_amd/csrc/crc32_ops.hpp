// GF(2) operator tables for the ENet CRC-32 (reflected polynomial 0xEDB88320).
//
// Reference semantics (jabuwu/rusty_enet, src/crc32.rs):
//   * CRC_TABLE (src/crc32.rs:1-34) is the byte-at-a-time table of the reflected
//     polynomial 0xEDB88320.  We never copy it: `sarwate` below is generated from
//     the polynomial at compile time (bitwise 8-step), and tests/test_oracle.py
//     checks it against the zlib-generated golden fixtures.
//   * crc32() (src/crc32.rs:39-47): reg = 0xFFFFFFFF; for every byte of the
//     concatenated slices  reg = (reg >> 8) ^ T[(reg ^ b) & 0xff];  result
//     (!reg).to_be(), i.e. bswap32(~reg) on little-endian hosts.
//
// The byte update is linear over GF(2):  reg' = M8(reg ^ b)  with
// M8(x) = (x >> 8) ^ T[x & 0xff].  Four byte steps on a little-endian word give
// reg' = M32(reg ^ w),  M32 = M8^4.  Every operator M32^n (advance the register
// over n zero words) is applied with four byte-indexed tables:
//     M32^n(x) = A0[x&0xff] ^ A1[(x>>8)&0xff] ^ A2[(x>>16)&0xff] ^ A3[x>>24],
//     Ak[b]    = M32^n(b << 8k).
// `op[lv]` holds those four tables for n = 2^lv words (lv = 0..kOpLevels-1).
// op[0][3] is the Sarwate table itself (M32(b<<24) = M8(b) = T[b]).
//
// `head_k[v]` = M8^{-v}(0xFFFFFFFF): injecting the 0xFFFFFFFF initial register
// into the first (partial) 32-bit word of a packet that starts v bytes into that
// word ("init injection").
#pragma once
#include <stdint.h>

namespace enet_crc {

constexpr uint32_t kReflectedPoly = 0xEDB88320u;
constexpr uint32_t kInitRegister = 0xFFFFFFFFu;
constexpr int kOpLevels = 9;  // M32^1 .. M32^256

struct OpTables {
  uint32_t sarwate[256];
  uint32_t op[kOpLevels][4][256];
  uint32_t head_k[4];
  uint8_t inv_top[256];  // inv_top[sarwate[b] >> 24] = b (see m8_inverse)
  uint32_t inv1[4][256];  // M32^-1 (back over one zero word), same four-table form
};

constexpr uint32_t sarwate_entry(uint32_t b) {
  uint32_t r = b;
  for (int i = 0; i < 8; ++i) r = (r & 1u) ? (r >> 1) ^ kReflectedPoly : (r >> 1);
  return r;
}

constexpr uint32_t apply_op(const uint32_t (&a)[4][256], uint32_t x) {
  return a[0][x & 0xffu] ^ a[1][(x >> 8) & 0xffu] ^ a[2][(x >> 16) & 0xffu] ^ a[3][x >> 24];
}

// Inverse of one zero-byte step M8.  The top byte of T[b] is a permutation of b
// for this polynomial, so the table index can be recovered from the output.
constexpr uint32_t m8_inverse(const uint32_t (&t)[256], uint32_t y) {
  for (uint32_t b = 0; b < 256; ++b) {
    if ((t[b] >> 24) == (y >> 24)) return ((y ^ t[b]) << 8) | b;
  }
  return 0;  // unreachable for the CRC-32 polynomial
}

constexpr OpTables make_op_tables() {
  OpTables t{};
  for (uint32_t b = 0; b < 256; ++b) t.sarwate[b] = sarwate_entry(b);
  // Level 0: M32 = four zero-byte steps.
  for (int k = 0; k < 4; ++k) {
    for (uint32_t b = 0; b < 256; ++b) {
      uint32_t r = b << (8 * k);
      for (int s = 0; s < 4; ++s) r = (r >> 8) ^ t.sarwate[r & 0xffu];
      t.op[0][k][b] = r;
    }
  }
  // Level lv: M32^(2^lv) = M32^(2^(lv-1)) o M32^(2^(lv-1)).
  for (int lv = 1; lv < kOpLevels; ++lv) {
    for (int k = 0; k < 4; ++k) {
      for (uint32_t b = 0; b < 256; ++b) {
        uint32_t x = b << (8 * k);
        x = apply_op(t.op[lv - 1], x);
        x = apply_op(t.op[lv - 1], x);
        t.op[lv][k][b] = x;
      }
    }
  }
  for (uint32_t b = 0; b < 256; ++b) t.inv_top[t.sarwate[b] >> 24] = (uint8_t)b;
  // M32^-1 = M8^-4, one byte step back at a time through inv_top (m8_inverse in O(1)).
  for (int k = 0; k < 4; ++k) {
    for (uint32_t b = 0; b < 256; ++b) {
      uint32_t y = b << (8 * k);
      for (int s = 0; s < 4; ++s) {
        const uint32_t i = t.inv_top[y >> 24];
        y = ((y ^ t.sarwate[i]) << 8) | i;
      }
      t.inv1[k][b] = y;
    }
  }
  uint32_t k = kInitRegister;
  t.head_k[0] = k;
  for (int v = 1; v < 4; ++v) {
    k = m8_inverse(t.sarwate, k);
    t.head_k[v] = k;
  }
  return t;
}

inline constexpr OpTables kOpTables = make_op_tables();

constexpr bool top_bytes_are_a_permutation() {
  bool seen[256] = {};
  for (uint32_t b = 0; b < 256; ++b) {
    const uint32_t top = kOpTables.sarwate[b] >> 24;
    if (seen[top]) return false;
    seen[top] = true;
  }
  return true;
}
static_assert(top_bytes_are_a_permutation(), "M8 must be invertible through the table's top bytes");

}  // namespace enet_crc
