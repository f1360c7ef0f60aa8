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
  hipMemcpy(d, h, n * L, hipMemcpyHostToDevice);
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  for (int i = 0; i < 5; ++i) enet_crc32_uniform_device(d, L, L, n, out, nullptr);
  hipDeviceSynchronize();
  const int it = 30;
  hipEventRecord(e0, 0);
  for (int i = 0; i < it; ++i) enet_crc32_uniform_device(d, L, L, n, out, nullptr);
  hipEventRecord(e1, 0); hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1);
  const double us = ms * 1000 / it;
  uint32_t o[4]; hipMemcpy(o, out, 16, hipMemcpyDeviceToHost);
  printf("%-28s %8.1f us  %7.1f GB/s  out0=%08x\n", VARIANT_NAME, us, n * L / (us * 1e3), o[0]);
#ifdef STAMPS
  // Per-wave cycle stamps of the last launch: ring wait (vmcnt), ring read (ds_read_b128),
  // combine, and the whole loop (s_memtime units).
  static unsigned long long st[5 * 8192];
  hipMemcpyFromSymbol(st, HIP_SYMBOL(enet_crc::g_stamp), sizeof(st));
  double sum[4] = {0, 0, 0, 0}, rt = 0;
  int nw = 0;
  for (int w = 0; w < 8192; ++w) {
    if (st[4 * w + 3] == 0) continue;
    ++nw;
    for (int j = 0; j < 4; ++j) sum[j] += st[4 * w + j];
    rt += st[32768 + w];
  }
  if (nw) printf("  in-kernel clock %.2f GHz (s_memtime / s_memrealtime x 100 MHz), loop %.1f us per wave\n",
                 sum[3] / rt * 0.1, rt / nw * 0.01);
  if (nw) printf("  stamps over %d waves: vm_wait %.0f  ds_read %.0f  combine %.0f  total %.0f cycles/wave (%.1f%% / %.1f%% / %.1f%%)\n",
                 nw, sum[0] / nw, sum[1] / nw, sum[2] / nw, sum[3] / nw, 100 * sum[0] / sum[3], 100 * sum[1] / sum[3],
                 100 * sum[2] / sum[3]);
#endif
  return 0;
}
