// LDS table layout and per-lane lookup addressing of the gfx950 kernels, shared by
// crc32_kernels.hip and its host-side check (tests/cpp/layout_check.cpp), which
// verifies on the CPU that every lane's addresses return the right operator entry
// and that each ds_read_b32 lookup is bank-conflict-free.
//
// Replicated block (64 KiB at LDS address 0): one 256-B row per byte value i,
//   row i = [ M32^32 set: dword t*8 + c | M32^1 set: dword 32 + t*8 + c ],
// t = table (register byte), c = copy (0..7).  A ds_read_b32 wave-instruction is
// serviced in two 32-lane groups; bank = dword address mod 32 = t*8 + c.  Lookup j of
// lane l reads table t = j ^ o with o = (l >> 3) & 3 and copy c = l & 7, so in every
// lane group the four octets read four different tables and the 32 lanes hit 32
// different banks whatever the register values are.  Each address is ONE v_perm_b32:
//   addr = (byte t of h) << 8 | lp.byte[j],   lp.byte[j] = set*128 + t*32 + c*4.
#pragma once
#include <stdint.h>

#include "crc32_geometry.hpp"
#include "crc32_ops.hpp"

namespace enet_crc {

constexpr uint32_t kRepCopies = 8;
constexpr uint32_t kRowDwords = 64;
constexpr uint32_t kRepDwords = 256 * kRowDwords;  // 64 KiB
constexpr uint32_t kSetM1Bytes = 128;               // byte offset of the M32^1 set inside a row
constexpr uint32_t kSarwateDword = 32 + 3 * 8;      // M32^1 table 3, copy 0 == the CRC table

constexpr int ilog2(int x) { return x <= 1 ? 0 : 1 + ilog2(x >> 1); }
constexpr int kMainLevel = ilog2(4 * kLanesPerPacket);  // M32^(4G) = M32^32
constexpr int kTreeLevels = ilog2(kLanesPerPacket);
constexpr uint32_t kTreeDword = kRepDwords;  // unreplicated tree operators M32^4, M32^8, M32^16
constexpr uint32_t kLdsDwords = kTreeDword + kTreeLevels * 1024;
// Layout of the register-ring kernel (no DMA ring, so LDS has room): a second replicated
// block at 64 KiB with the first two tree levels (set 0: M32^4, set 1: M32^8; same row
// format and per-lane addressing as the main block, so the masked tree lookups are
// bank-conflict-free too), then M32^16 unreplicated (one lane in 8 looks it up).
constexpr uint32_t kTreeRepDword = kRepDwords;
constexpr uint32_t kTree16Dword = 2 * kRepDwords;
constexpr uint32_t kRegsLdsDwords = kTree16Dword + 1024;
static_assert(kMainLevel < kOpLevels, "operator level");
static_assert(kRepCopies * 4 == 32, "8 copies x 4 tables cover the 32 banks of a ds_read_b32 lane group");

// v_perm_b32(s0, s1, sel): byte k of the result is byte sel.k of {s0:s1} (0-3 from s1,
// 4-7 from s0); 0x0C gives 0x00.  Only the selector values used here are modelled
// on the host.
ENET_HD uint32_t perm_b32(uint32_t s0, uint32_t s1, uint32_t sel) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_perm(s0, s1, sel);
#else
  const uint64_t v = ((uint64_t)s0 << 32) | s1;
  uint32_t r = 0;
  for (int k = 0; k < 4; ++k) {
    const uint32_t b = (sel >> (8 * k)) & 0xffu;
    const uint32_t byte = b < 8 ? (uint32_t)(v >> (8 * b)) & 0xffu : 0u;
    r |= byte << (8 * k);
  }
  return r;
#endif
}

// Per-lane constants of the replicated-table lookups.
struct Lookup {
  uint32_t lp;      // byte j: byte offset inside a row of this lane's copy of M32^32 table t
  uint32_t lp1;     // the same for the M32^1 set
  uint32_t sel[4];  // v_perm selectors: byte0 <- lp byte j, byte1 <- h byte t (the row)
};

ENET_HD Lookup make_lookup(uint32_t lane) {
  const uint32_t oct = (lane >> 3) & 3u, copy = lane & 7u;
  Lookup lk{};
  for (uint32_t j = 0; j < 4; ++j) {
    const uint32_t t = j ^ oct;
    lk.lp |= (copy * 4u + 32u * t) << (8u * j);
    lk.lp1 |= (kSetM1Bytes + copy * 4u + 32u * t) << (8u * j);
    lk.sel[j] = 0x0C0C0000u | ((4u + t) << 8) | j;
  }
  return lk;
}

// LDS byte address of lookup j for register value h (lp = lk.lp or lk.lp1).
ENET_HD uint32_t lookup_addr(uint32_t h, uint32_t lp, const Lookup& lk, int j) { return perm_b32(h, lp, lk.sel[j]); }

// The LDS image fill_lds() writes (dword index -> value), as a host function.
inline void host_lds_image(uint32_t* lds) {
  const OpTables& T = kOpTables;
  for (uint32_t x = 0; x < kLdsDwords; ++x) lds[x] = 0;
  for (uint32_t tab = 0; tab < 4; ++tab)
    for (uint32_t i = 0; i < 256; ++i)
      for (uint32_t c = 0; c < kRepCopies; ++c) {
        lds[i * kRowDwords + tab * kRepCopies + c] = T.op[kMainLevel][tab][i];
        lds[i * kRowDwords + kSetM1Bytes / 4 + tab * kRepCopies + c] = T.op[0][tab][i];
      }
  for (int set = 0; set < kTreeLevels; ++set)
    for (uint32_t r = 0; r < 1024; ++r) lds[kTreeDword + set * 1024 + r] = T.op[set + 2][r >> 8][r & 255];
}

// The register-ring kernel's LDS image (kRegsLdsDwords).
inline void host_lds_image_regs(uint32_t* lds) {
  const OpTables& T = kOpTables;
  for (uint32_t x = 0; x < kRegsLdsDwords; ++x) lds[x] = 0;
  for (uint32_t tab = 0; tab < 4; ++tab)
    for (uint32_t i = 0; i < 256; ++i)
      for (uint32_t c = 0; c < kRepCopies; ++c) {
        lds[i * kRowDwords + tab * kRepCopies + c] = T.op[kMainLevel][tab][i];
        lds[i * kRowDwords + kSetM1Bytes / 4 + tab * kRepCopies + c] = T.op[0][tab][i];
        lds[kTreeRepDword + i * kRowDwords + tab * kRepCopies + c] = T.op[2][tab][i];
        lds[kTreeRepDword + i * kRowDwords + kSetM1Bytes / 4 + tab * kRepCopies + c] = T.op[3][tab][i];
      }
  for (uint32_t r = 0; r < 1024; ++r) lds[kTree16Dword + r] = T.op[4][r >> 8][r & 255];
}

}  // namespace enet_crc
