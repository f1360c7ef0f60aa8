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
  return 0;
}
