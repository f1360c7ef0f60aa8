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

// Wait for the sequence word, then sum 348 data words (a 1392-B datagram) and answer
// {seq, sum} in pinned host memory.
__global__ void spin_data(volatile unsigned* flag, unsigned want, const unsigned* data, unsigned* host_ack,
                          unsigned long long limit) {
  const unsigned long long t0 = wall_clock64();
  while (true) {
    unsigned v;
    asm volatile("global_load_dword %0, %1, off sc0 sc1\n\ts_waitcnt vmcnt(0)" : "=v"(v) : "v"(flag) : "memory");
    if (v == want) break;
    if (wall_clock64() - t0 > limit) break;
  }
  // All six loads of a lane in flight together (one wait): words lane + 64 i.
  unsigned w[6];
  const unsigned* a[6];
  for (int i = 0; i < 6; ++i) {
    const unsigned k = threadIdx.x + 64u * i;
    a[i] = data + (k < 348 ? k : 0);
  }
  asm volatile(
      "global_load_dword %0, %6, off sc0 sc1\n\t"
      "global_load_dword %1, %7, off sc0 sc1\n\t"
      "global_load_dword %2, %8, off sc0 sc1\n\t"
      "global_load_dword %3, %9, off sc0 sc1\n\t"
      "global_load_dword %4, %10, off sc0 sc1\n\t"
      "global_load_dword %5, %11, off sc0 sc1\n\t"
      "s_waitcnt vmcnt(0)"
      : "=&v"(w[0]), "=&v"(w[1]), "=&v"(w[2]), "=&v"(w[3]), "=&v"(w[4]), "=&v"(w[5])
      : "v"(a[0]), "v"(a[1]), "v"(a[2]), "v"(a[3]), "v"(a[4]), "v"(a[5])
      : "memory");
  unsigned part = 0;
  for (int i = 0; i < 6; ++i) part += threadIdx.x + 64u * i < 348 ? w[i] : 0u;
  for (int o = 32; o >= 1; o >>= 1) part += __shfl_xor(part, o, 64);
  if (threadIdx.x == 0) {
    asm volatile("global_store_dword %0, %1, off sc0 sc1\n\ts_waitcnt vmcnt(0)" ::"v"(host_ack + 1), "v"(part) : "memory");
    asm volatile("global_store_dword %0, %1, off sc0 sc1\n\ts_waitcnt vmcnt(0)" ::"v"(host_ack), "v"(want) : "memory");
  }
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
  for (int fence = 0; fence < 2; ++fence) {
  best = 1e9; sum = 0;
  hp[0] = 0;
  for (int i = 1; i <= 200; ++i) {
    hipLaunchKernelGGL(spin_until, dim3(1), dim3(64), 0, 0, (volatile unsigned*)d, (unsigned)i, dack, 100000000ull);
    for (volatile int k = 0; k < 200000; ++k) {}  // let the kernel start spinning
    const auto t0 = std::chrono::steady_clock::now();
    __atomic_store_n((unsigned*)hp, (unsigned)i, __ATOMIC_RELEASE);
    if (fence) __builtin_ia32_sfence();  // drain the write-combining buffer of the BAR mapping
    while (__atomic_load_n(&ack[0], __ATOMIC_ACQUIRE) != (unsigned)i) {}
    const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
    hipDeviceSynchronize();
    if (i > 10) { best = us < best ? us : best; sum += us; }
  }
  printf("round trip host->VRAM flag->GPU->host ack (%s): best %.2f us, mean %.2f us\n",
         fence ? "sfence after the store" : "no fence", best, sum / 190);
  fflush(stdout);
  }
  // A 1392-B datagram + sequence word written into VRAM through the BAR (then sfence); the
  // wave sees the sequence word, sums the datagram's words from VRAM and answers in
  // pinned host memory: the data path a VRAM mailbox would use.
  {
    unsigned* data = d + 16;  // 64 B past the flag
    unsigned src[348];
    for (int k = 0; k < 348; ++k) src[k] = 0x9E3779B9u * (unsigned)(k + 1);
    unsigned want_sum = 0;
    for (int k = 0; k < 348; ++k) want_sum += src[k];
    best = 1e9; sum = 0;
    int bad = 0;
    hp[0] = 0;
    ack[0] = 0;
    for (int i = 1; i <= 200; ++i) {
      hipLaunchKernelGGL(spin_data, dim3(1), dim3(64), 0, 0, (volatile unsigned*)d, (unsigned)i, data, dack,
                         100000000ull);
      for (volatile int k = 0; k < 200000; ++k) {}
      src[0] = 0x9E3779B9u + (unsigned)i;
      const unsigned ws = want_sum - 0x9E3779B9u + src[0];
      const auto t0 = std::chrono::steady_clock::now();
      memcpy((void*)data, src, sizeof src);
      __builtin_ia32_sfence();
      __atomic_store_n((unsigned*)hp, (unsigned)i, __ATOMIC_RELEASE);
      __builtin_ia32_sfence();
      while (__atomic_load_n(&ack[0], __ATOMIC_ACQUIRE) != (unsigned)i) {}
      const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
      hipDeviceSynchronize();
      bad += ack[1] != ws;
      if (i > 10) { best = us < best ? us : best; sum += us; }
    }
    printf("1392-B datagram host->VRAM (memcpy + sfence) -> GPU sum -> host: best %.2f us, mean %.2f us, "
           "wrong sums %d\n", best, sum / 190, bad);
    fflush(stdout);
  }
  // The same datagram test with flag and data in pinned host memory (the current
  // mailbox): the wave reads the datagram across PCIe.
  {
    unsigned* hbox = nullptr;
    hipHostMalloc((void**)&hbox, 4096, hipHostMallocMapped | hipHostMallocCoherent);
    unsigned* dbox = nullptr;
    hipHostGetDevicePointer((void**)&dbox, hbox, 0);
    unsigned src[348];
    for (int k = 0; k < 348; ++k) src[k] = 0x7F4A7C15u * (unsigned)(k + 1);
    unsigned want_sum = 0;
    for (int k = 0; k < 348; ++k) want_sum += src[k];
    double b2 = 1e9, s2 = 0;
    int bad = 0;
    hbox[0] = 0;
    ack[0] = 0;
    for (int i = 1; i <= 200; ++i) {
      hipLaunchKernelGGL(spin_data, dim3(1), dim3(64), 0, 0, (volatile unsigned*)dbox, (unsigned)i, dbox + 16, dack,
                         100000000ull);
      for (volatile int k = 0; k < 200000; ++k) {}
      src[0] = 0x7F4A7C15u + (unsigned)i;
      const unsigned ws = want_sum - 0x7F4A7C15u + src[0];
      const auto t0 = std::chrono::steady_clock::now();
      memcpy(hbox + 16, src, sizeof src);
      __atomic_store_n(hbox, (unsigned)i, __ATOMIC_RELEASE);
      while (__atomic_load_n(&ack[0], __ATOMIC_ACQUIRE) != (unsigned)i) {}
      const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
      hipDeviceSynchronize();
      bad += ack[1] != ws;
      if (i > 10) { b2 = us < b2 ? us : b2; s2 += us; }
    }
    printf("1392-B datagram in pinned host memory -> GPU sum -> host: best %.2f us, mean %.2f us, wrong sums %d\n",
           b2, s2 / 190, bad);
    fflush(stdout);
  }
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
