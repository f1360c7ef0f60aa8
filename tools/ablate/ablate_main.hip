// Ablation harness (tooling, not product): times launch_uniform() of a patched copy of
// rusty_enet_amd/csrc/crc32_kernels.hip (see tools/ablate/run.sh) on 1M x 1200 B.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include "variant.hip"
#include "../../rusty_enet_amd/csrc/enet_crc_abi.hip"

int main(int argc, char** argv) {
  const uint64_t n = 1 << 20, L = argc > 1 ? atoi(argv[1]) : 1200;
  uint8_t* d; uint32_t* out;
  hipMalloc(&d, n * L); hipMalloc(&out, n * 4);
  uint8_t* h = (uint8_t*)malloc(n * L);
  uint64_t x = 88172645463325252ull;
  for (uint64_t i = 0; i < n * L; i += 8) { x ^= x << 13; x ^= x >> 7; x ^= x << 17; memcpy(h + i, &x, 8); }
  if (getenv("ABLATE_CONST")) memset(h, 0x5a, n * L);  // constant bytes (HBM power depends on data)
  hipMemcpy(d, h, n * L, hipMemcpyHostToDevice);
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  for (int i = 0; i < 5; ++i) enet_crc32_uniform_device(d, L, L, n, out, nullptr);
  hipDeviceSynchronize();
  const int it = 30;
  hipEventRecord(e0, 0);
  for (int i = 0; i < it; ++i) enet_crc32_uniform_device(d, L, L, n, out, nullptr);
  hipEventRecord(e1, 0); hipEventSynchronize(e1);
  if (hipDeviceSynchronize() != hipSuccess || hipGetLastError() != hipSuccess) {
    fprintf(stderr, "%s: HIP error, stopping\n", VARIANT_NAME);
    exit(2);
  }
  float ms; hipEventElapsedTime(&ms, e0, e1);
  const double us = ms * 1000 / it;
  uint32_t o[4]; hipMemcpy(o, out, 16, hipMemcpyDeviceToHost);
  printf("%-28s %8.1f us  %7.1f GB/s  out0=%08x\n", VARIANT_NAME, us, n * L / (us * 1e3), o[0]);
#ifdef STAMPS
  // Per-wave cycle stamps of the last launch: ring wait (vmcnt), ring read (ds_read_b128),
  // combine, and the whole loop (s_memtime units).
  static unsigned long long st[6 * 8192];
  hipMemcpyFromSymbol(st, HIP_SYMBOL(enet_crc::g_stamp), sizeof(st));
  double sum[4] = {0, 0, 0, 0}, rt = 0;
  int nw = 0;
  for (int w = 0; w < 8192; ++w) {
    if (st[4 * w + 3] == 0) continue;
    ++nw;
    for (int j = 0; j < 4; ++j) sum[j] += st[4 * w + j];
    rt += st[32768 + w];
  }
  {
    unsigned long long s0 = ~0ull, s1 = 0, e1 = 0, e0 = ~0ull, dmin = ~0ull, dmax = 0;
    for (int w = 0; w < 8192; ++w) {
      if (st[4 * w + 3] == 0) continue;
      const unsigned long long a = st[40960 + w], d = st[32768 + w], e = a + d;
      s0 = a < s0 ? a : s0; s1 = a > s1 ? a : s1; e0 = e < e0 ? e : e0; e1 = e > e1 ? e : e1;
      dmin = d < dmin ? d : dmin; dmax = d > dmax ? d : dmax;
    }
    if (nw) printf("  loop start spread %.1f us, end spread %.1f us (first end %.1f, last end %.1f us after first start), loop min %.1f max %.1f us\n",
                   (s1 - s0) * 0.01, (e1 - e0) * 0.01, (e0 - s0) * 0.01, (e1 - s0) * 0.01, dmin * 0.01, dmax * 0.01);
  }
  {
    // Wave end times grouped by XCD (workgroup b runs on XCD b % 8).
    unsigned long long s0 = ~0ull;
    for (int w = 0; w < 8192; ++w)
      if (st[4 * w + 3] && st[40960 + w] < s0) s0 = st[40960 + w];
    double sum_x[8] = {0}, max_x[8] = {0}, min_x[8] = {1e30, 1e30, 1e30, 1e30, 1e30, 1e30, 1e30, 1e30};
    int n_x[8] = {0};
    for (int w = 0; w < 8192; ++w) {
      if (st[4 * w + 3] == 0) continue;
      const int x = (w / 16) % 8;
      const double e = (st[40960 + w] + st[32768 + w] - s0) * 0.01;
      sum_x[x] += e; ++n_x[x];
      max_x[x] = e > max_x[x] ? e : max_x[x];
      min_x[x] = e < min_x[x] ? e : min_x[x];
    }
    printf("  end time by XCD (mean/min/max us):");
    for (int x = 0; x < 8; ++x) if (n_x[x]) printf(" %d:%.0f/%.0f/%.0f", x, sum_x[x] / n_x[x], min_x[x], max_x[x]);
    printf("\n");
  }
  if (nw) printf("  in-kernel clock %.2f GHz (s_memtime / s_memrealtime x 100 MHz), loop %.1f us per wave\n",
                 sum[3] / rt * 0.1, rt / nw * 0.01);
  if (nw) printf("  stamps over %d waves: vm_wait %.0f  ds_read %.0f  combine %.0f  total %.0f cycles/wave (%.1f%% / %.1f%% / %.1f%%)\n",
                 nw, sum[0] / nw, sum[1] / nw, sum[2] / nw, sum[3] / nw, 100 * sum[0] / sum[3], 100 * sum[1] / sum[3],
                 100 * sum[2] / sum[3]);
#endif
  return 0;
}
