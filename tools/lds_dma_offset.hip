// Probe (tooling): where does global_load_lds_dwordx4 with a nonzero immediate offset put
// its data in LDS?  One wave loads 16 B per lane from src + 256 (the immediate) with the LDS
// destination pointer at byte 1024 of a 4-KiB LDS array, then dumps the whole array.  Prints
// the LDS byte offset at which lane 0's 16 bytes landed: 1024 if the immediate applies to the
// global address only, 1280 if it applies to both addresses.  Everything stays inside the
// 4-KiB array and the 2-KiB source buffer either way.
//   hipcc --offload-arch=gfx950 -O2 -o tools/lds_dma_offset tools/lds_dma_offset.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

typedef __attribute__((address_space(3))) void LdsVoid;

__global__ __launch_bounds__(64) void probe(const uint32_t* src, uint32_t* dump) {
  __shared__ __attribute__((aligned(16))) uint32_t lds[1024];
  for (int i = threadIdx.x; i < 1024; i += 64) lds[i] = 0xDEADBEEFu;
  __syncthreads();
  const char* g = reinterpret_cast<const char*>(src) + 16 * threadIdx.x;
  __builtin_amdgcn_global_load_lds((const void*)g, (LdsVoid*)((char*)lds + 1024), 16, 256, 0);
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();
  for (int i = threadIdx.x; i < 1024; i += 64) dump[i] = lds[i];
}

int main() {
  uint32_t h[512];
  for (int i = 0; i < 512; ++i) h[i] = 0x10000u + (uint32_t)i;  // word i of the source
  uint32_t *src = nullptr, *dump = nullptr;
  if (hipMalloc(&src, sizeof(h)) != hipSuccess || hipMalloc(&dump, 4096) != hipSuccess) return 2;
  if (hipMemcpy(src, h, sizeof(h), hipMemcpyHostToDevice) != hipSuccess) return 2;
  hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, src, dump);
  uint32_t d[1024];
  if (hipMemcpy(d, dump, 4096, hipMemcpyDeviceToHost) != hipSuccess) return 3;
  // Lane 0 loads source bytes 256..271 = words 64..67.
  int at = -1;
  for (int i = 0; i < 1024; ++i)
    if (d[i] == 0x10000u + 64u) {
      at = 4 * i;
      break;
    }
  printf("lane 0's data landed at LDS byte %d (1024: offset on the global address only; 1280: on both)\n", at);
  return at == 1024 || at == 1280 ? 0 : 1;
}
