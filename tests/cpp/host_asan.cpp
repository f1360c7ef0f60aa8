// Host-side code under AddressSanitizer + UndefinedBehaviorSanitizer (SURVEY.md §5;
// `make asan` builds and runs it, tests/test_asan.py calls make).  Covers the pure host
// functions the C ABI exports or uses (rusty_enet_amd/csrc/crc32_host.hpp:
// split_bounds = enet_crc_shard_bounds, slot_adjust_checksum = enet_crc32_slot_adjust,
// combine_checksums = enet_crc32_combine, plan_stage_chunk = the staging chunks of
// enet_crc32_ragged_host) against the C oracle, and the oracle itself (the CRC
// restatement of src/crc32.rs and the range-coder restatement of src/c/compress.rs,
// round trips and output-limit exits).  Exit status 0 = every check passed.
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <random>
#include <vector>

#include "../../rusty_enet_amd/csrc/crc32_host.hpp"

extern "C" {
typedef struct {
  const uint8_t* data;
  size_t len;
} oracle_iov;
uint32_t oracle_crc32(const uint8_t* p, size_t n);
uint32_t oracle_crc32_iov(const oracle_iov* bufs, size_t n);
void oracle_crc32_ragged(const uint8_t* base, const uint64_t* offsets, const uint32_t* lengths, uint64_t count,
                         uint32_t* out);
int oracle_crc32_uniform_mt(const uint8_t* base, uint64_t stride, uint32_t length, uint64_t count, uint32_t* out,
                            int threads);
int oracle_enet_verify(uint8_t* datagram, size_t length, size_t header_size, uint32_t slot_value);
size_t oracle_range_compress(const oracle_iov* bufs, size_t nbufs, size_t in_limit, uint8_t* out, size_t out_limit);
size_t oracle_range_decompress(const uint8_t* in, size_t in_len, uint8_t* out, size_t out_limit);
}

using namespace enet_crc;

static int g_fail = 0;
static long g_checks = 0;
#define CHECK(c)                                                         \
  do {                                                                   \
    ++g_checks;                                                          \
    if (!(c)) {                                                          \
      if (g_fail++ < 20) fprintf(stderr, "%s:%d: %s\n", __FILE__, __LINE__, #c); \
    }                                                                    \
  } while (0)

static std::vector<uint8_t> bytes(std::mt19937_64& r, size_t n) {
  std::vector<uint8_t> v(n);
  for (auto& b : v) b = (uint8_t)r();
  return v;
}

static void test_split_bounds(std::mt19937_64& r) {
  for (int t = 0; t < 400; ++t) {
    const uint64_t count = r() % 1000;
    const uint32_t n = 1 + (uint32_t)(r() % 70);
    std::vector<uint32_t> len(count);
    for (auto& l : len) l = (r() % 5 == 0) ? 0 : (uint32_t)(r() % (t % 3 == 0 ? 70000 : 1500));
    std::vector<uint64_t> b(n + 1);
    const bool even = t % 7 == 0;
    split_bounds(even ? nullptr : len.data(), count, n, b.data());
    CHECK(b[0] == 0 && b[n] == count);
    uint64_t total = 0, maxl = 0;
    for (auto l : len) total += l, maxl = l > maxl ? l : maxl;
    for (uint32_t k = 0; k < n; ++k) {
      CHECK(b[k] <= b[k + 1]);
      if (even) {
        CHECK(b[k + 1] - b[k] <= count / n + 1);
      } else {
        uint64_t bytes_k = 0;
        for (uint64_t i = b[k]; i < b[k + 1]; ++i) bytes_k += len[i];
        CHECK(bytes_k <= total / n + maxl + 1);  // within one packet of an even share
      }
    }
  }
}

static void test_slot_adjust(std::mt19937_64& r) {
  for (int t = 0; t < 600; ++t) {
    const size_t h = (r() & 1) ? 8 : 6;  // header_size (protocol.rs:1412-1415)
    const size_t len = h + (size_t)(t % 50 == 0 ? r() % 70000 : r() % 4096);
    std::vector<uint8_t> d = bytes(r, len);
    const uint32_t u = (uint32_t)r(), v = (uint32_t)r();
    memcpy(d.data() + h - 4, &u, 4);
    const uint32_t cu = oracle_crc32(d.data(), len);
    memcpy(d.data() + h - 4, &v, 4);
    const uint32_t cv = oracle_crc32(d.data(), len);
    CHECK(slot_adjust_checksum(cu, u, v, (uint32_t)(len - h)) == cv);
    // the receive check as the oracle does it (protocol.rs:1470-1502): slot = checksum
    memcpy(d.data() + h - 4, &cv, 4);
    std::vector<uint8_t> e = d;
    CHECK(oracle_enet_verify(e.data(), len, h, v) == 1);
  }
}

static void test_combine(std::mt19937_64& r) {
  const uint8_t a8[8] = {1, 2, 3, 4, 5, 6, 7, 8}, b8[8] = {8, 7, 6, 5, 4, 3, 2, 1};
  CHECK(oracle_crc32(a8, 8) == 3314076223u);  // src/crc32.rs:52
  CHECK(combine_checksums(oracle_crc32(a8, 8), oracle_crc32(b8, 8), 8) == 1712484799u);  // :54-55
  for (int t = 0; t < 800; ++t) {
    const size_t la = r() % 3000, lb = (t % 40 == 0) ? r() % 100000 : r() % 3000;
    std::vector<uint8_t> buf = bytes(r, la + lb);
    const uint32_t ca = oracle_crc32(buf.data(), la), cb = oracle_crc32(buf.data() + la, lb);
    CHECK(combine_checksums(ca, cb, lb) == oracle_crc32(buf.data(), la + lb));
  }
  // associativity far past any buffer (ladder below 2^34 bytes, matrix powering above)
  for (int t = 0; t < 200; ++t) {
    const uint32_t a = (uint32_t)r(), b = (uint32_t)r(), c = (uint32_t)r();
    // lengths >= 1 (a random checksum is only consistent with a non-empty part), sum < 2^64
    const uint64_t nb = (r() >> (t % 60 + 1)) | 1, nc = (r() >> (t % 61 + 2)) | 1;
    CHECK(combine_checksums(combine_checksums(a, b, nb), c, nc) == combine_checksums(a, combine_checksums(b, c, nc),
                                                                                       nb + nc));
  }
}

static void test_stage_chunks(std::mt19937_64& r) {
  for (int t = 0; t < 300; ++t) {
    const uint64_t count = 1 + r() % 3000;
    std::vector<uint64_t> off(count);
    std::vector<uint32_t> len(count);
    uint64_t pos = r() % 16;
    for (uint64_t i = 0; i < count; ++i) {
      len[i] = (uint32_t)(r() % (t % 5 == 0 ? 20000 : 1500));
      if (t % 4 == 0) {
        off[i] = r() % 2000000;  // any order, overlaps
      } else {
        off[i] = pos;
        pos += len[i] + (t % 3 ? 0 : r() % 64);
      }
    }
    const uint64_t max_bytes = 1 + r() % 200000, max_packets = 1 + r() % 700;
    std::vector<uint8_t> seen(count, 0);
    uint64_t p = 0;
    while (p < count) {
      const StageChunk c = plan_stage_chunk(off.data(), len.data(), count, p, max_bytes, max_packets);
      CHECK(c.end > p && c.end <= count && c.end - p <= max_packets);
      CHECK(c.lo_al % 4 == 0);
      CHECK(c.end - p == 1 || c.span <= max_bytes + 3);
      for (uint64_t i = p; i < c.end; ++i) {
        seen[i]++;
        CHECK(off[i] >= c.lo_al && off[i] + len[i] <= c.lo_al + c.span);  // staged copy holds the packet
      }
      p = c.end;
    }
    for (uint64_t i = 0; i < count; ++i) CHECK(seen[i] == 1);
  }
}

static void test_oracle(std::mt19937_64& r) {
  // ragged and multi-threaded uniform drivers agree with single calls
  const uint64_t n = 3000;
  std::vector<uint8_t> data = bytes(r, n * 1201 + 8);
  std::vector<uint64_t> off(n);
  std::vector<uint32_t> len(n);
  for (uint64_t i = 0; i < n; ++i) off[i] = i * 1201 + (r() % 3), len[i] = (uint32_t)(r() % 1199);
  std::vector<uint32_t> out(n), mt(n);
  oracle_crc32_ragged(data.data(), off.data(), len.data(), n, out.data());
  for (uint64_t i = 0; i < n; ++i) CHECK(out[i] == oracle_crc32(data.data() + off[i], len[i]));
  CHECK(oracle_crc32_uniform_mt(data.data(), 1201, 1200, n, mt.data(), 8) == 0);
  for (uint64_t i = 0; i < n; ++i) CHECK(mt[i] == oracle_crc32(data.data() + i * 1201, 1200));
  // range coder: round trips over compressible and random bytes, multi-slice inputs,
  // and the output-limit exits (compress.rs:79-81, the limit checks of enc_put)
  for (int t = 0; t < 300; ++t) {
    const size_t m = 1 + r() % 4000;
    std::vector<uint8_t> in(m);
    for (auto& b : in) b = (t & 1) ? (uint8_t)r() : (uint8_t)(r() % 6);
    // two non-empty slices (an empty slice is read as one 0 byte: compress.rs:119-122)
    const size_t cut = m > 1 ? 1 + r() % (m - 1) : m;
    oracle_iov iov[2] = {{in.data(), cut}, {in.data() + cut, m - cut}};
    const size_t nio = m > 1 ? 2 : 1;
    std::vector<uint8_t> comp(2 * m + 64), back(m + 16);
    const size_t cs = oracle_range_compress(iov, nio, m, comp.data(), comp.size());
    if (cs) {
      const size_t ds = oracle_range_decompress(comp.data(), cs, back.data(), m);
      CHECK(ds == m && memcmp(back.data(), in.data(), m) == 0);
      CHECK(oracle_range_decompress(comp.data(), cs, back.data(), m > 1 ? m - 1 : 0) == 0 || m == 1);
    }
    const size_t lim = r() % (m + 1);
    std::vector<uint8_t> small(lim + 1);
    const size_t cl = oracle_range_compress(iov, nio, m, small.data(), lim);
    CHECK(cl <= lim);
  }
}

int main() {
  std::mt19937_64 r(0x454E4554);
  test_split_bounds(r);
  test_slot_adjust(r);
  test_combine(r);
  test_stage_chunks(r);
  test_oracle(r);
  printf("host_asan: %ld checks, %d failed\n", g_checks, g_fail);
  return g_fail ? 1 : 0;
}
