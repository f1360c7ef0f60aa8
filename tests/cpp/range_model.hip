// Host run of the range-coder KERNEL code (rusty_enet_amd/csrc/range_coder.hip,
// whose coder functions are __host__ __device__) against the CPU oracle
// (oracle/range_coder_oracle.c).  No GPU: only the host side of this TU runs.
// Checks compressed bytes + sizes, round trips, output-limit failures and
// decompression of arbitrary (non-coder) byte strings.  Prints "bad=<n>".
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <random>
#include <vector>

#include "../../rusty_enet_amd/csrc/range_coder.hip"

extern "C" {
typedef struct oracle_iov {
  const uint8_t* data;
  size_t len;
} oracle_iov;
size_t oracle_range_compress(const oracle_iov* bufs, size_t nbufs, size_t in_limit, uint8_t* out, size_t out_limit);
size_t oracle_range_decompress(const uint8_t* in, size_t in_len, uint8_t* out, size_t out_limit);
}

using enet_crc::Model;
using enet_crc::Sym;

int main() {
  std::vector<Sym> arena(4096);
  memset((void*)arena.data(), getenv("RC_GARBAGE") ? 0xAB : 0, arena.size() * sizeof(Sym));
  Model m;
  m.a = arena.data();
  std::mt19937_64 rng(0x454E4554);
  long bad = 0, cases = 0;
  std::vector<uint8_t> in, o1, o2, d1, d2;
  for (int t = 0; t < 6000; ++t) {
    const int kind = t % 6;
    size_t n = (t < 64) ? (size_t)t : (size_t)(rng() % (kind == 5 ? 9000 : 1500));
    in.resize(n);
    for (size_t i = 0; i < n; ++i) {
      uint64_t r = rng();
      switch (kind) {
        case 0: in[i] = (uint8_t)r; break;                        // incompressible
        case 1: in[i] = (uint8_t)(r & 3); break;                  // 2-bit alphabet
        case 2: in[i] = 0; break;                                 // zeros: rescale paths
        case 3: in[i] = (uint8_t)("ENet reliable command "[i % 22]); break;
        case 4: in[i] = (uint8_t)((r % 16) == 0 ? r >> 8 : 7); break;  // skewed
        default: in[i] = (uint8_t)(r % 40); break;                // long: arena resets
      }
    }
    // output limit: generous, or tight (= input size, the protocol's limit), or tiny
    size_t lim = (t % 3 == 0) ? n : (t % 3 == 1) ? 2 * n + 64 : (size_t)(rng() % 12);
    o1.assign(lim + 1, 0xAA);
    o2.assign(lim + 1, 0xAA);
    oracle_iov one = {in.data(), n};
    size_t s1 = oracle_range_compress(&one, 1, n, o1.data(), lim);
    size_t s2 = enet_crc::compress_one(m, in.data(), (uint32_t)n, o2.data(), (uint32_t)lim);
    ++cases;
    if (s1 != s2 || memcmp(o1.data(), o2.data(), s1) != 0) {
      if (bad < 5) printf("compress mismatch t=%d kind=%d n=%zu lim=%zu: %zu vs %zu\n", t, kind, n, lim, s1, s2);
      ++bad;
      continue;
    }
    if (s1 == 0) continue;
    // decompress with an exact, a generous and a short output limit
    for (size_t dl : {n, n + 100, n / 2}) {
      d1.assign(dl + 1, 0x55);
      d2.assign(dl + 1, 0x55);
      size_t r1 = oracle_range_decompress(o1.data(), s1, d1.data(), dl);
      size_t r2 = enet_crc::decompress_one(m, o2.data(), (uint32_t)s1, d2.data(), (uint32_t)dl);
      ++cases;
      if (r1 != r2 || memcmp(d1.data(), d2.data(), r1) != 0 || (dl >= n && (r1 != n || memcmp(d1.data(), in.data(), n)))) {
        if (bad < 5) printf("decompress mismatch t=%d n=%zu dl=%zu: %zu vs %zu\n", t, n, dl, r1, r2);
        ++bad;
      }
    }
  }
  // arbitrary byte strings fed to the decoder (malformed streams: error returns must agree)
  for (int t = 0; t < 4000; ++t) {
    size_t n = 1 + rng() % 64;
    in.resize(n);
    for (auto& b : in) b = (uint8_t)rng();
    size_t dl = 1 + rng() % 4096;
    d1.assign(dl, 0);
    d2.assign(dl, 0);
    size_t r1 = oracle_range_decompress(in.data(), n, d1.data(), dl);
    size_t r2 = enet_crc::decompress_one(m, in.data(), (uint32_t)n, d2.data(), (uint32_t)dl);
    ++cases;
    if (r1 != r2 || memcmp(d1.data(), d2.data(), r1) != 0) {
      if (bad < 5) printf("garbage mismatch t=%d n=%zu: %zu vs %zu\n", t, n, r1, r2);
      ++bad;
    }
  }
  printf("cases=%ld bad=%ld\n", cases, bad);
  return bad != 0;
}
