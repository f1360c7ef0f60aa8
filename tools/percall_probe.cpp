// Per-call latency of enet_crc32_iov from C (no Python): one 1392-B datagram (the
// reference's default MTU) per call, every per-call mode, checked against a host
// Sarwate CRC.  Prints best / median / mean microseconds per call.
//   g++ -O2 -Iinclude tools/percall_probe.cpp -Lrusty_enet_amd/lib -lenet_crc_amd -o tools/percall_probe
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdint>
#include <vector>

#include "enet_crc_amd.h"

static uint32_t host_crc(const uint8_t* p, size_t n) {  // src/crc32.rs:39-47, for the check only
  static uint32_t t[256];
  if (!t[1])
    for (uint32_t b = 0; b < 256; ++b) {
      uint32_t c = b;
      for (int k = 0; k < 8; ++k) c = (c >> 1) ^ ((c & 1) ? 0xEDB88320u : 0u);
      t[b] = c;
    }
  uint32_t r = 0xFFFFFFFFu;
  for (size_t i = 0; i < n; ++i) r = (r >> 8) ^ t[(r ^ p[i]) & 0xff];
  return __builtin_bswap32(~r);
}

int main(int argc, char** argv) {
  const size_t len = argc > 1 ? (size_t)atoi(argv[1]) : 1392;
  enet_crc_ctx* ctx = nullptr;
  if (enet_crc_ctx_create(0, &ctx) != 0) {
    printf("no context\n");
    return 1;
  }
  std::vector<uint8_t> d(len);
  const char* names[3] = {"copy", "zerocopy", "persistent"};
  const int modes[3] = {ENET_CRC_PERCALL_COPY, ENET_CRC_PERCALL_ZEROCOPY, ENET_CRC_PERCALL_PERSISTENT};
  int bad = 0;
  for (int m = 0; m < 3; ++m) {
    if (enet_crc_ctx_set_percall_mode(ctx, modes[m]) != 0) return 1;
    std::vector<double> us;
    for (int i = 0; i < 3000; ++i) {
      for (size_t k = 0; k < len; ++k) d[k] = (uint8_t)(k * 31 + i);
      enet_crc_iov v{d.data(), len};
      uint32_t crc = 0;
      const auto t0 = std::chrono::steady_clock::now();
      const int st = enet_crc32_iov(ctx, &v, 1, &crc);
      const double t = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
      if (st != 0 || crc != host_crc(d.data(), len)) ++bad;
      if (i >= 100) us.push_back(t);
    }
    std::sort(us.begin(), us.end());
    double sum = 0;
    for (double x : us) sum += x;
    printf("%-10s %zu B: best %.2f us, median %.2f us, mean %.2f us\n", names[m], len, us.front(), us[us.size() / 2],
           sum / us.size());
    fflush(stdout);
  }
  enet_crc_ctx_destroy(ctx);
  printf("wrong results: %d\n", bad);
  return bad ? 1 : 0;
}
