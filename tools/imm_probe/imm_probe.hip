// Probe (tooling): does the immediate offset of global_load_lds_dwordx4 also move the LDS
// destination?  One wave loads 16 B per lane from src + 16 lane + 256 (offset:256) into an
// LDS buffer cleared to 0xFFFFFFFF, and dumps the buffer.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
typedef __attribute__((address_space(3))) void LdsVoid;
__global__ void probe(const uint32_t* src, uint32_t* out) {
  __shared__ __attribute__((aligned(16))) uint32_t s[1024];
  for (int i = threadIdx.x; i < 1024; i += 64) s[i] = 0xFFFFFFFFu;
  __syncthreads();
  __builtin_amdgcn_global_load_lds((const void*)(src + 4 * threadIdx.x), (LdsVoid*)(s + 128), 16, 256, 0);
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();
  for (int i = threadIdx.x; i < 1024; i += 64) out[i] = s[i];
}
int main() {
  uint32_t h[2048], o[1024];
  for (int i = 0; i < 2048; ++i) h[i] = (uint32_t)i;
  uint32_t *ds, *dout;
  if (hipMalloc(&ds, sizeof h) || hipMalloc(&dout, sizeof o)) return 1;
  hipMemcpy(ds, h, sizeof h, hipMemcpyHostToDevice);
  probe<<<1, 64>>>(ds, dout);
  if (hipDeviceSynchronize() != hipSuccess) return 2;
  hipMemcpy(o, dout, sizeof o, hipMemcpyDeviceToHost);
  int first = -1, last = -1;
  for (int i = 0; i < 1024; ++i)
    if (o[i] != 0xFFFFFFFFu) { if (first < 0) first = i; last = i; }
  printf("written LDS dwords %d..%d; s[%d] = %u (src dword), s[128] = %u\n", first, last, first, first >= 0 ? o[first] : 0u, o[128]);
  printf("LDS offset applied: %s\n", first == 128 + 64 ? "yes (dest moved by 256 B)" : first == 128 ? "no" : "other");
  return 0;
}
