// Probe: can the host write device memory directly (fine-grained VRAM through the PCIe
// BAR), and how long does a GPU wave take to see such a write?  Prints one line per step.
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstring>

__global__ void spin_until(volatile unsigned* flag, unsigned want, unsigned* host_ack, unsigned long long limit) {
  const unsigned long long t0 = wall_clock64();
  while (true) {
    unsigned v;
    asm volatile("global_load_dword %0, %1, off sc0 sc1\n\ts_waitcnt vmcnt(0)" : "=v"(v) : "v"(flag) : "memory");
    if (v == want) break;
    if (wall_clock64() - t0 > limit) break;
  }
  asm volatile("global_store_dword %0, %1, off sc0 sc1\n\ts_waitcnt vmcnt(0)" ::"v"(host_ack), "v"(want) : "memory");
}

int main() {
  unsigned* d = nullptr;
  hipError_t e = hipExtMallocWithFlags((void**)&d, 4096, hipDeviceMallocFinegrained);
  printf("alloc fine-grained: %s\n", hipGetErrorString(e));
  if (e != hipSuccess) return 1;
  hipPointerAttribute_t a{};
  e = hipPointerGetAttributes(&a, d);
  printf("attrs: %s type=%d hostPointer=%p devicePointer=%p\n", hipGetErrorString(e), (int)a.type, a.hostPointer, a.devicePointer);
  fflush(stdout);
  // host write through the same pointer (SVM: valid only if the VRAM is host-mapped)
  volatile unsigned* hp = (volatile unsigned*)d;
  hp[0] = 0;
  printf("host wrote device memory\n");
  fflush(stdout);
  unsigned* ack = nullptr;
  hipHostMalloc((void**)&ack, 64, hipHostMallocMapped | hipHostMallocCoherent);
  ack[0] = 0;
  unsigned* dack = nullptr;
  hipHostGetDevicePointer((void**)&dack, ack, 0);
  double best = 1e9, sum = 0;
  for (int i = 1; i <= 200; ++i) {
    hipLaunchKernelGGL(spin_until, dim3(1), dim3(64), 0, 0, (volatile unsigned*)d, (unsigned)i, dack, 100000000ull);
    for (volatile int k = 0; k < 200000; ++k) {}  // let the kernel start spinning
    const auto t0 = std::chrono::steady_clock::now();
    __atomic_store_n((unsigned*)hp, (unsigned)i, __ATOMIC_RELEASE);
    while (__atomic_load_n(&ack[0], __ATOMIC_ACQUIRE) != (unsigned)i) {}
    const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
    hipDeviceSynchronize();
    if (i > 10) { best = us < best ? us : best; sum += us; }
  }
  printf("round trip host->VRAM flag->GPU->host ack: best %.2f us, mean %.2f us\n", best, sum / 190);
  // same with the flag in pinned host memory
  unsigned* hflag = nullptr;
  hipHostMalloc((void**)&hflag, 64, hipHostMallocMapped | hipHostMallocCoherent);
  unsigned* dflag = nullptr;
  hipHostGetDevicePointer((void**)&dflag, hflag, 0);
  hflag[0] = 0;
  best = 1e9; sum = 0;
  for (int i = 1; i <= 200; ++i) {
    hipLaunchKernelGGL(spin_until, dim3(1), dim3(64), 0, 0, (volatile unsigned*)dflag, 1000u + i, dack, 100000000ull);
    for (volatile int k = 0; k < 200000; ++k) {}
    const auto t0 = std::chrono::steady_clock::now();
    __atomic_store_n(hflag, 1000u + i, __ATOMIC_RELEASE);
    while (__atomic_load_n(&ack[0], __ATOMIC_ACQUIRE) != 1000u + i) {}
    const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
    hipDeviceSynchronize();
    if (i > 10) { best = us < best ? us : best; sum += us; }
  }
  printf("round trip host-memory flag->GPU->host ack: best %.2f us, mean %.2f us\n", best, sum / 190);
  return 0;
}
