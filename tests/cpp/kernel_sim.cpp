// Host-side model of the gfx950 kernel's arithmetic (crc32_kernels.hip), lane by
// lane, checked against the oracle restatement of src/crc32.rs.  Test
// infrastructure only: it exercises the GF(2) operator tables
// (rusty_enet_amd/csrc/crc32_ops.hpp), the end-aligned stream decomposition, the
// head masking / init injection and the fixed-shift combine tree for every lane
// count the kernel template allows, without a GPU.  kExt models the LDS-DMA kernels'
// trailing-byte handling: the packet runs to the next 4-byte boundary with the bytes
// past its end masked to zero, and the last word's shift stops z bytes short
// (finish_word: M8^(4-z) y from the M32^1 tables, instead of M32 y).  kA16 (with kExt)
// models 16-B-aligned chunks: the packet runs on to the next 16-B boundary, u = 0..3 more
// zero words, and the combined value goes back over them with M32^-1 before finish_word.
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <random>
#include <vector>

#include "../../rusty_enet_amd/csrc/crc32_geometry.hpp"
#include "../../rusty_enet_amd/csrc/crc32_ops.hpp"

extern "C" {
struct oracle_iov { const uint8_t* data; size_t len; };
uint32_t oracle_crc32(const uint8_t* p, size_t n);
const uint32_t* oracle_crc_table(void);
}

using namespace enet_crc;
static const OpTables& T = kOpTables;

static uint32_t op(int lv, uint32_t x) { return apply_op(T.op[lv], x); }

template <int G, bool kExt = false, bool kA16 = false>
static uint32_t model(const uint8_t* buf, uint64_t s, uint64_t len) {
  static_assert(!kA16 || kExt, "16-B chunks only in the extended form");
  const uint64_t z = kExt && len ? (4 - ((s + len) & 3)) & 3 : 0;
  const uint64_t sa = s, ea = s + len, top = sa & ~3ull, a1x = kExt ? (ea + z) : (ea & ~3ull);
  const uint64_t a1 = kA16 && len ? (a1x + 15) & ~15ull : a1x;
  const uint32_t u = (uint32_t)((a1 - a1x) >> 2);  // zero words past the packet's last word
  // Word at byte address a (a >= top): the packet's bytes, zeros past its end (kExt).
  auto word_at = [&](uint64_t a) {
    uint32_t w = 0;
    memcpy(&w, buf + a, 4);
    if (kExt && a >= ea) return 0u;
    if (kExt && a + 4 > ea) w &= 0xFFFFFFFFu >> (8 * (a + 4 - ea));
    return w;
  };
  const uint64_t nwords = (a1 - top) >> 2;
  constexpr int kMain = __builtin_ctz(4 * G);
  uint32_t reg = kInitRegister;
  if (nwords > 0) {
    const uint64_t nchunks = (nwords + 3) >> 2;
    const int64_t nsteps = (int64_t)((nchunks + G - 1) / G);
    uint32_t h[G][4];
    for (int k = 0; k < G; ++k) {
      const int64_t c = k + (int64_t)G * (nsteps - 1);
      for (int j = 0; j < 4; ++j) {
        const int64_t rel = (int64_t)(a1 - top) - 16 * (c + 1) + 4 * j;
        uint32_t w = 0;
        if (rel >= 0) w = word_at(top + rel);
        if (rel == 0) {
          const uint32_t v = (uint32_t)(sa - top);
          w = (w & (0xFFFFFFFFu << (8 * v))) ^ T.head_k[v];
        }
        h[k][j] = w;
      }
      for (int64_t i = nsteps - 2; i >= 0; --i) {
        uint32_t q[4];
        for (int j = 0; j < 4; ++j) q[j] = word_at(a1 - 16 * (k + G * i + 1) + 4 * j);
        for (int j = 0; j < 4; ++j) h[k][j] = op(kMain, h[k][j]) ^ q[j];
      }
    }
    uint32_t y[G];
    for (int k = 0; k < G; ++k) y[k] = op(0, op(0, op(0, h[k][0]) ^ h[k][1]) ^ h[k][2]) ^ h[k][3];
    for (int l = 1; (1 << l) <= G; ++l) {
      const int d = 1 << (l - 1);
      uint32_t t[G];
      for (int k = 0; k < G; ++k) t[k] = op(l + 1, y[k]);
      for (int k = 0; k + d < G; ++k) y[k] ^= t[k + d];
    }
    if (kExt) {
      // finish_word: M8^(4-z)(y) = M32(y << 8z) ^ (y >> (32 - 8z)): the bytes shifted out
      // of the register unchanged, the rest through the ordinary M32 tables.
      const uint32_t zz = (uint32_t)z;
      uint32_t yy = y[0];
      for (uint32_t i = 0; i < u; ++i) yy = apply_op(T.inv1, yy);
      reg = op(0, zz ? yy << (8 * zz) : yy) ^ (zz ? yy >> (32 - 8 * zz) : 0u);
    } else {
      reg = op(0, y[0]);
    }
  }
  if constexpr (!kExt) {
    for (uint64_t b = (a1 > sa ? a1 : sa); b < ea; ++b) reg = (reg >> 8) ^ T.sarwate[(reg ^ buf[b]) & 0xffu];
  }
  return __builtin_bswap32(~reg);
}

// crc32_uniform_lines_kernel, lane by lane: one round of 8 back-to-back packets of L bytes
// (L a multiple of 16) at the 128-B aligned offset r0; group g reads the round's lines
// [g L / 128, (g+1) L / 128), lane k chunk m of each line (lines_lane, crc32_geometry.hpp).
// Returns the number of wrong checksums; -1 if a lane would read outside the round.
static int model_lines(const uint8_t* buf, uint64_t r0, uint32_t L) {
  const int nsl = (int)((L + 127) / 128);
  uint32_t h[64][4] = {}, kept[64][4] = {};
  for (uint32_t lane = 0; lane < 64; ++lane) {
    const LinesLane ll = lines_lane(L, nsl, lane / 8, lane % 8);
    for (int s = 0; s < nsl; ++s) {
      uint32_t w[4] = {0, 0, 0, 0};
      if (!(s == 0 && ll.dummy0)) {
        const int64_t off = ll.off0 + 128 * s;
        if (off < 0 || off + 16 > 8 * (int64_t)L) return -1;
        memcpy(w, buf + r0 + off, 16);
      }
      if (s < 2) {
        if (ll.keep[s]) memcpy(kept[lane], w, 16);
        w[0] = (w[0] & ll.am[s]) ^ ll.xm[s];
        for (int j = 1; j < 4; ++j) w[j] &= ll.am[s];
      }
      for (int j = 0; j < 4; ++j) h[lane][j] = s == 0 ? w[j] : op(5, h[lane][j]) ^ w[j];
    }
  }
  int bad = 0;
  for (uint32_t g = 0; g < 8; ++g) {
    uint32_t y[8];
    for (uint32_t k = 0; k < 8; ++k) {
      const uint32_t lane = 8 * g + k;
      const LinesLane ll = lines_lane(L, nsl, g, k);
      uint32_t hh[4];
      for (int j = 0; j < 4; ++j) hh[j] = ll.lo ? op(5, h[lane][j]) ^ kept[ll.src4 / 4][j] : h[lane][j];
      y[k] = op(0, op(0, op(0, hh[0]) ^ hh[1]) ^ hh[2]) ^ hh[3];
    }
    for (int l = 1; l <= 3; ++l) {
      const int d = 1 << (l - 1);
      uint32_t t[8];
      for (int k = 0; k < 8; ++k) t[k] = op(l + 1, y[k]);
      for (int k = 0; k + d < 8; ++k) y[k] ^= t[k + d];
    }
    const uint32_t crc = __builtin_bswap32(~op(0, y[0]));
    bad += crc != oracle_crc32(buf + r0 + g * L, L);
  }
  return bad;
}

int main() {
  int bad = 0;
  const uint32_t* ot = oracle_crc_table();
  for (int b = 0; b < 256; ++b) bad += T.sarwate[b] != ot[b];
  for (int b = 0; b < 256; ++b) bad += T.op[0][3][b] != ot[b];  // M32(b<<24) == T[b]
  // head_k[v] = M8^{-v}(~0): M8^v(head_k[v]) must give back ~0.
  for (int v = 0; v < 4; ++v) {
    uint32_t r = T.head_k[v];
    for (int i = 0; i < v; ++i) r = (r >> 8) ^ T.sarwate[r & 0xff];
    bad += r != 0xFFFFFFFFu;
  }
  // M32^-1 undoes M32.
  for (uint32_t x : {0u, 1u, 0x80000000u, 0xDEADBEEFu, 0x12345678u, 0xFFFFFFFFu}) bad += apply_op(T.inv1, op(0, x)) != x;
  if (bad) { printf("table mismatch %d\n", bad); return 1; }
  std::mt19937_64 g(12345);
  std::vector<uint8_t> buf(1 << 19);
  for (auto& x : buf) x = (uint8_t)g();
  long cases = 0;
  for (int it = 0; it < 60000; ++it) {
    const uint64_t s = g() % 4096;
    const uint64_t len = it < 6000 ? (uint64_t)(it % 600) : g() % (it % 11 == 0 ? 300000 : 3000);
    if (s + len > buf.size()) continue;
    const uint32_t want = oracle_crc32(buf.data() + s, len);
    // model<64, true>: the wave-per-packet kernel (crc32_wave_dma_kernel, 1-KiB steps);
    // model<4, true>: the 16-packet ragged kernel (crc32_ragged16_kernel, 64-B steps).
    // model<8, true, true>: the 8-lane ragged kernel with 16-B-aligned chunks.
    const uint32_t got[8] = {model<2>(buf.data(), s, len), model<4>(buf.data(), s, len),
                             model<8>(buf.data(), s, len), model<16>(buf.data(), s, len),
                             model<8, true>(buf.data(), s, len), model<64, true>(buf.data(), s, len),
                             model<4, true>(buf.data(), s, len), model<8, true, true>(buf.data(), s, len)};
    for (uint32_t v : got) {
      if (v != want) {
        if (bad < 10) printf("mismatch s=%llu len=%llu want %08x got %08x\n", (unsigned long long)s,
                             (unsigned long long)len, want, v);
        ++bad;
      }
    }
    ++cases;
  }
  // The whole-line kernel: every 16-B multiple length it takes (5..14 lines per round slot).
  for (uint32_t L = 528; L <= 1792; L += 16) {
    for (int r = 0; r < 6; ++r) {
      const int e = model_lines(buf.data(), 128 * (g() % 2048), L);
      if (e != 0) {
        if (bad < 10) printf("lines model L=%u: %d\n", L, e);
        bad += e < 0 ? 1 : e;
      }
      ++cases;
    }
  }
  printf("cases=%ld bad=%d\n", cases, bad);
  return bad ? 1 : 0;
}
