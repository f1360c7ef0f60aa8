// Host check of the kernels' LDS table layout and per-lane lookup addressing
// (rusty_enet_amd/csrc/crc32_layout.hpp, the same code the gfx950 kernels run):
//   1. for every lane and random register values, the 4 lookups of each replicated
//      set XOR to the operator (M32^32 or M32^1) applied to the register;
//   2. every ds_read_b32 lookup instruction is bank-conflict-free: within each of the
//      two 32-lane groups, no two lanes hit one bank at different dword addresses;
//   3. the CRC table read by the byte steps (kSarwateDword) is the reference table;
//   4. the same for the register-ring kernel's replicated tree block (M32^4, M32^8).
// Test infrastructure only.
#include <cstdint>
#include <cstdio>
#include <random>
#include <vector>

#include "../../rusty_enet_amd/csrc/crc32_layout.hpp"

using namespace enet_crc;

int main() {
  std::vector<uint32_t> lds(kLdsDwords);
  host_lds_image(lds.data());
  const OpTables& T = kOpTables;
  std::mt19937_64 rng(0x454E4554);
  long bad_value = 0, conflicts = 0, checks = 0;
  Lookup lk[64];
  for (uint32_t l = 0; l < 64; ++l) lk[l] = make_lookup(l);
  for (int trial = 0; trial < 20000; ++trial) {
    uint32_t h[64];
    for (auto& x : h) x = (uint32_t)rng();
    if (trial < 256)  // also registers whose bytes collide across lanes
      for (uint32_t l = 0; l < 64; ++l) h[l] = (uint32_t)trial * 0x01010101u;
    for (int set = 0; set < 2; ++set) {
      const int level = set == 0 ? kMainLevel : 0;
      for (int j = 0; j < 4; ++j) {
        for (int grp = 0; grp < 2; ++grp) {
          int64_t bank_addr[32];
          for (auto& a : bank_addr) a = -1;
          for (uint32_t l = 32 * grp; l < 32 * grp + 32; ++l) {
            const uint32_t a = lookup_addr(h[l], set ? lk[l].lp1 : lk[l].lp, lk[l], j);
            const uint32_t dw = a / 4, bank = dw % 32;
            if (a % 4 != 0 || dw >= kRepDwords) ++bad_value;
            if (bank_addr[bank] >= 0 && bank_addr[bank] != dw) ++conflicts;
            bank_addr[bank] = dw;
          }
        }
      }
      for (uint32_t l = 0; l < 64; ++l) {
        uint32_t x = 0;
        for (int j = 0; j < 4; ++j) x ^= lds[lookup_addr(h[l], set ? lk[l].lp1 : lk[l].lp, lk[l], j) / 4];
        ++checks;
        if (x != apply_op(T.op[level], h[l])) ++bad_value;
      }
    }
  }
  for (uint32_t i = 0; i < 256; ++i)
    if (lds[i * kRowDwords + kSarwateDword] != T.sarwate[i]) ++bad_value;
  // 4. The register-ring kernel's replicated tree block (combine_tree_rep): M32^4 (set 0)
  //    and M32^8 (set 1) at kTreeRepDword, same addressing, conflict-free; and its main
  //    block is the same as above.
  std::vector<uint32_t> rl(kRegsLdsDwords);
  host_lds_image_regs(rl.data());
  for (uint32_t x = 0; x < kRepDwords; ++x)
    if (rl[x] != lds[x]) ++bad_value;
  for (int trial = 0; trial < 20000; ++trial) {
    uint32_t h[64];
    for (auto& x : h) x = (uint32_t)rng();
    for (int set = 0; set < 2; ++set) {
      for (int j = 0; j < 4; ++j)
        for (int grp = 0; grp < 2; ++grp) {
          int64_t bank_addr[32];
          for (auto& a : bank_addr) a = -1;
          for (uint32_t l = 32 * grp; l < 32 * grp + 32; ++l) {
            const uint32_t dw = kTreeRepDword + lookup_addr(h[l], set ? lk[l].lp1 : lk[l].lp, lk[l], j) / 4;
            const uint32_t bank = dw % 32;
            if (bank_addr[bank] >= 0 && bank_addr[bank] != dw) ++conflicts;
            bank_addr[bank] = dw;
          }
        }
      for (uint32_t l = 0; l < 64; ++l) {
        uint32_t x = 0;
        for (int j = 0; j < 4; ++j)
          x ^= rl[kTreeRepDword + lookup_addr(h[l], set ? lk[l].lp1 : lk[l].lp, lk[l], j) / 4];
        ++checks;
        if (x != apply_op(T.op[set ? 3 : 2], h[l])) ++bad_value;
      }
    }
  }
  for (uint32_t r = 0; r < 1024; ++r)
    if (rl[kTree16Dword + r] != T.op[4][r >> 8][r & 255]) ++bad_value;
  std::printf("checks=%ld bad=%ld conflicts=%ld lds_bytes=%u\n", checks, bad_value, conflicts, kLdsDwords * 4);
  return bad_value == 0 && conflicts == 0 ? 0 : 1;
}
