// Read-bandwidth probe (tooling, not product): what does a plain global_load_dwordx4
// stream reach on this MI355X at the occupancy the CRC kernels use (one 1024-thread
// workgroup per CU, 144 KiB LDS), versus higher occupancy?  Each lane XOR-reduces
// 16-byte loads; the result is stored so nothing is dead code.
//   hipcc --offload-arch=gfx950 -O3 -o tools/read_probe tools/read_probe.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

// Pattern A: each wave reads contiguous 1 KiB pieces (lane l: bytes 16l..16l+15).
// Pattern B: CRC-kernel shape: 8 groups x 8 lanes, group g reads 128 B of packet (p0+g)
//            at stride `stride`, step i -> offset 128 i within the packet.
template <int UNROLL, int LDS_KB, bool kPatternB, int kNT = 0>
__global__ __launch_bounds__(1024) void probe(const uint8_t* __restrict__ buf, uint64_t bytes, uint64_t stride,
                                              uint32_t* __restrict__ out) {
  __shared__ uint32_t lds[LDS_KB * 256 + 1];
  if (LDS_KB) lds[threadIdx.x] = threadIdx.x;
  __syncthreads();
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t wave = (uint64_t)blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64;
  const uint64_t nwaves = (uint64_t)gridDim.x * (blockDim.x / 64);
  u32x4 acc = {0, 0, 0, 0};
  if (!kPatternB) {
    const uint64_t pieces = bytes / 1024;
    for (uint64_t p = wave * UNROLL; p < pieces; p += nwaves * UNROLL) {
      u32x4 v[UNROLL];
#pragma unroll
      for (int u = 0; u < UNROLL; ++u) {
        const uint64_t q = p + u < pieces ? p + u : p;
        if (kNT) v[u] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(buf + q * 1024 + lane * 16));
        else v[u] = *reinterpret_cast<const u32x4*>(buf + q * 1024 + lane * 16);
      }
#pragma unroll
      for (int u = 0; u < UNROLL; ++u) acc ^= v[u];
    }
  } else {
    const uint32_t g = lane / 8, k = lane % 8;
    const uint64_t npk = bytes / stride;
    const uint64_t steps = (stride + 127) / 128;  // assumes stride % 16 == 0
    for (uint64_t r = wave; r * 8 < npk; r += nwaves) {
      const uint64_t pkt = r * 8 + g < npk ? r * 8 + g : npk - 1;
      const uint8_t* base = buf + pkt * stride;
      for (uint64_t i = 0; i < steps; i += UNROLL) {
        u32x4 v[UNROLL];
#pragma unroll
        for (int u = 0; u < UNROLL; ++u) {
          uint64_t off = (i + u) * 128 + k * 16;
          off = off + 16 <= stride ? off : 0;
          if (kNT) v[u] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(base + off));
          else v[u] = *reinterpret_cast<const u32x4*>(base + off);
        }
#pragma unroll
        for (int u = 0; u < UNROLL; ++u) acc ^= v[u];
      }
    }
  }
  if (LDS_KB) acc.x ^= lds[(threadIdx.x * 7) & 1023];
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc.x ^ acc.y ^ acc.z ^ acc.w;
}

// Pattern A through LDS-DMA (global_load_lds_dwordx4): each wave owns a ring of R
// 1-KiB LDS slots; loads land in LDS, lanes read them back with ds_read_b128.
// Pattern B consumed as a ring: slot s of round r is consumed, then slot s of round
// r+1 is issued (one load per slot, spread over the round), with `work` dependent
// VALU ops per slot standing in for the CRC arithmetic.  kBurst instead issues all
// of round r+1's loads at the start of round r (double buffer).
template <int NS, int LOOK, bool kNoMem = false, int LDSKB = 144>
__global__ __launch_bounds__(1024) void probe_deep(const uint8_t* __restrict__ buf, uint64_t bytes, uint64_t stride,
                                                   uint32_t* __restrict__ out, int work) {
  __shared__ uint32_t lds[LDSKB * 256];
  lds[threadIdx.x] = threadIdx.x;
  __syncthreads();
  const uint32_t lane = threadIdx.x & 63, g = lane / 8, k = lane % 8;
  const uint64_t wave = (uint64_t)blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64;
  const uint64_t nwaves = (uint64_t)gridDim.x * (blockDim.x / 64);
  const uint64_t npk = bytes / stride;
  auto addr = [&](uint64_t r, int s) -> const u32x4* {
    uint64_t pkt = r * 8 + g;
    if (pkt >= npk) pkt = npk - 1;
    uint64_t off = (uint64_t)s * 128 + k * 16;
    off = off + 16 <= stride ? off : 0;
    if (kNoMem) return reinterpret_cast<const u32x4*>(buf + ((pkt * 16 + off) & 1023));
    return reinterpret_cast<const u32x4*>(buf + pkt * stride + off);
  };
  u32x4 acc = {0, 0, 0, 0};
  u32x4 q[LOOK][NS];
  uint64_t r = wave;
#pragma unroll
  for (int l = 0; l < LOOK; ++l)
#pragma unroll
    for (int s = 0; s < NS; ++s) { q[l][s] = *addr(r + l * nwaves, s); __builtin_amdgcn_sched_barrier(0); }
  for (; r * 8 < npk; r += LOOK * nwaves) {
#pragma unroll
    for (int l = 0; l < LOOK; ++l) {
#pragma unroll
      for (int s = 0; s < NS; ++s) {
        uint32_t x = q[l][s].x ^ q[l][s].y ^ q[l][s].z ^ q[l][s].w;
        for (int t = 0; t < work; ++t) x = __builtin_amdgcn_perm(x, x * 3u, 0x05040100u) + t;
        acc.x ^= x;
        q[l][s] = *addr(r + (l + LOOK) * nwaves, s);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc.x ^ acc.y ^ acc.z ^ acc.w;
}

template <int NS, int LOOK, bool kNoMem = false, int LDSKB = 144>
static void run_deep(const char* name, const uint8_t* d, uint64_t bytes, uint32_t* out, int blocks, int work, int threads = 1024) {
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  for (int w = 0; w < 3; ++w) hipLaunchKernelGGL((probe_deep<NS, LOOK, kNoMem, LDSKB>), dim3(blocks), dim3(threads), 0, 0, d, bytes, 1200, out, work);
  CHECK(hipDeviceSynchronize());
  const int iters = 20;
  CHECK(hipEventRecord(e0, 0));
  for (int w = 0; w < iters; ++w) hipLaunchKernelGGL((probe_deep<NS, LOOK, kNoMem, LDSKB>), dim3(blocks), dim3(threads), 0, 0, d, bytes, 1200, out, work);
  CHECK(hipEventRecord(e1, 0));
  CHECK(hipEventSynchronize(e1));
  float ms = 0;
  CHECK(hipEventElapsedTime(&ms, e0, e1));
  const double us = ms * 1000.0 / iters;
  printf("%-40s work=%3d  %8.1f us  %7.1f GB/s\n", name, work, us, bytes / (us * 1e3));
}

template <int NS, bool kBurst>
__global__ __launch_bounds__(1024) void probe_ring(const uint8_t* __restrict__ buf, uint64_t bytes, uint64_t stride,
                                                   uint32_t* __restrict__ out, int work) {
  __shared__ uint32_t lds[144 * 256];
  lds[threadIdx.x] = threadIdx.x;
  __syncthreads();
  const uint32_t lane = threadIdx.x & 63, g = lane / 8, k = lane % 8;
  const uint64_t wave = (uint64_t)blockIdx.x * 16 + threadIdx.x / 64;
  const uint64_t nwaves = (uint64_t)gridDim.x * 16;
  const uint64_t npk = bytes / stride;
  auto addr = [&](uint64_t r, int s) -> const u32x4* {
    uint64_t pkt = r * 8 + g;
    if (pkt >= npk) pkt = npk - 1;
    uint64_t off = (uint64_t)s * 128 + k * 16;
    off = off + 16 <= stride ? off : 0;
    return reinterpret_cast<const u32x4*>(buf + pkt * stride + off);
  };
  u32x4 acc = {0, 0, 0, 0};
  u32x4 q[NS], q2[NS];
  uint64_t r = wave;
#pragma unroll
  for (int s = 0; s < NS; ++s) { q[s] = *addr(r, s); __builtin_amdgcn_sched_barrier(0); }
  for (; r * 8 < npk; r += nwaves) {
    if (kBurst) {
#pragma unroll
      for (int s = 0; s < NS; ++s) { q2[s] = *addr(r + nwaves, s); __builtin_amdgcn_sched_barrier(0); }
    }
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      uint32_t x = q[s].x ^ q[s].y ^ q[s].z ^ q[s].w;
      for (int t = 0; t < work; ++t) x = __builtin_amdgcn_perm(x, x * 3u, 0x05040100u) + t;
      acc.x ^= x;
      if (!kBurst) { q[s] = *addr(r + nwaves, s); __builtin_amdgcn_sched_barrier(0); }
    }
    if (kBurst) {
#pragma unroll
      for (int s = 0; s < NS; ++s) q[s] = q2[s];
    }
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc.x ^ acc.y ^ acc.z ^ acc.w;
}

template <int NS, bool kBurst>
static void run_ring(const char* name, const uint8_t* d, uint64_t bytes, uint32_t* out, int blocks, int work) {
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  for (int w = 0; w < 3; ++w) hipLaunchKernelGGL((probe_ring<NS, kBurst>), dim3(blocks), dim3(1024), 0, 0, d, bytes, 1200, out, work);
  CHECK(hipDeviceSynchronize());
  const int iters = 20;
  CHECK(hipEventRecord(e0, 0));
  for (int w = 0; w < iters; ++w) hipLaunchKernelGGL((probe_ring<NS, kBurst>), dim3(blocks), dim3(1024), 0, 0, d, bytes, 1200, out, work);
  CHECK(hipEventRecord(e1, 0));
  CHECK(hipEventSynchronize(e1));
  float ms = 0;
  CHECK(hipEventElapsedTime(&ms, e0, e1));
  const double us = ms * 1000.0 / iters;
  printf("%-40s work=%3d  %8.1f us  %7.1f GB/s\n", name, work, us, bytes / (us * 1e3));
}

template <int R>
__global__ __launch_bounds__(1024) void probe_dma(const uint8_t* __restrict__ buf, uint64_t bytes, uint64_t work,
                                                  uint32_t* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) uint8_t ring[16][R][1024];
  const uint32_t lane = threadIdx.x & 63, w = threadIdx.x / 64;
  const uint64_t wave = (uint64_t)blockIdx.x * 16 + w;
  const uint64_t nwaves = (uint64_t)gridDim.x * 16;
  const uint64_t pieces = bytes / 1024;
  u32x4 acc = {0, 0, 0, 0};
  for (uint64_t p = wave * R; p < pieces; p += nwaves * R) {
#pragma unroll
    for (int u = 0; u < R; ++u) {
      const uint64_t q = p + u < pieces ? p + u : p;
      __builtin_amdgcn_global_load_lds((const void*)(buf + q * 1024 + lane * 16), (__attribute__((address_space(3))) void*)&ring[w][u][0], 16, 0, 0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
    for (int u = 0; u < R; ++u) {
      u32x4 v = *reinterpret_cast<const u32x4*>(&ring[w][u][lane * 16]);
      uint32_t x = v.x ^ v.y ^ v.z ^ v.w;
      for (uint64_t t = 0; t < work; ++t) x = __builtin_amdgcn_perm(x, x * 3u, 0x05040100u) + (uint32_t)t;
      acc.x ^= x;
    }
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc.x ^ acc.y ^ acc.z ^ acc.w;
}

// One 1-KiB LDS slot per wave: ds_read_b128 the landed slot into registers, issue the
// next slot's DMA into the same buffer, then compute on the registers while it flies.
template <int LDSKB_EXTRA>
__global__ __launch_bounds__(1024) void probe_dma1(const uint8_t* __restrict__ buf, uint64_t bytes, uint64_t work,
                                                   uint32_t* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) uint8_t ring[16][1024];
  __shared__ uint32_t pad[LDSKB_EXTRA * 256];
  pad[threadIdx.x] = threadIdx.x;
  const uint32_t lane = threadIdx.x & 63, w = threadIdx.x / 64;
  const uint64_t wave = (uint64_t)blockIdx.x * 16 + w;
  const uint64_t nwaves = (uint64_t)gridDim.x * 16;
  const uint64_t pieces = bytes / 1024;
  u32x4 acc = {0, 0, 0, 0};
  uint64_t p = wave;
  if (p < pieces)
    __builtin_amdgcn_global_load_lds((const void*)(buf + p * 1024 + lane * 16), (__attribute__((address_space(3))) void*)&ring[w][0], 16, 0, 0);
  for (; p < pieces; p += nwaves) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    u32x4 v = *reinterpret_cast<const u32x4*>(&ring[w][lane * 16]);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    const uint64_t pn = p + nwaves < pieces ? p + nwaves : p;
    __builtin_amdgcn_global_load_lds((const void*)(buf + pn * 1024 + lane * 16), (__attribute__((address_space(3))) void*)&ring[w][0], 16, 0, 0);
    uint32_t x = v.x ^ v.y ^ v.z ^ v.w;
    for (uint64_t t = 0; t < work; ++t) x = __builtin_amdgcn_perm(x, x * 3u, 0x05040100u) + (uint32_t)t;
    acc.x ^= x;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc.x ^ acc.y ^ acc.z ^ acc.w ^ pad[(threadIdx.x * 3) & 255];
}

template <int LDSKB_EXTRA>
static void run_dma1(const char* name, const uint8_t* d, uint64_t bytes, uint32_t* out, int blocks, uint64_t work) {
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  for (int w = 0; w < 3; ++w) hipLaunchKernelGGL((probe_dma1<LDSKB_EXTRA>), dim3(blocks), dim3(1024), 0, 0, d, bytes, work, out);
  CHECK(hipDeviceSynchronize());
  const int iters = 20;
  CHECK(hipEventRecord(e0, 0));
  for (int w = 0; w < iters; ++w) hipLaunchKernelGGL((probe_dma1<LDSKB_EXTRA>), dim3(blocks), dim3(1024), 0, 0, d, bytes, work, out);
  CHECK(hipEventRecord(e1, 0));
  CHECK(hipEventSynchronize(e1));
  float ms = 0;
  CHECK(hipEventElapsedTime(&ms, e0, e1));
  const double us = ms * 1000.0 / iters;
  printf("%-40s work=%3d  %8.1f us  %7.1f GB/s\n", name, (int)work, us, bytes / (us * 1e3));
}

template <int R>
static void run_dma(const char* name, const uint8_t* d, uint64_t bytes, uint32_t* out, int blocks, uint64_t work = 0) {
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  for (int w = 0; w < 3; ++w) hipLaunchKernelGGL((probe_dma<R>), dim3(blocks), dim3(1024), 0, 0, d, bytes, work, out);
  CHECK(hipDeviceSynchronize());
  const int iters = 20;
  CHECK(hipEventRecord(e0, 0));
  for (int w = 0; w < iters; ++w) hipLaunchKernelGGL((probe_dma<R>), dim3(blocks), dim3(1024), 0, 0, d, bytes, work, out);
  CHECK(hipEventRecord(e1, 0));
  CHECK(hipEventSynchronize(e1));
  float ms = 0;
  CHECK(hipEventElapsedTime(&ms, e0, e1));
  const double us = ms * 1000.0 / iters;
  printf("%-40s work=%3d  %8.1f us  %7.1f GB/s\n", name, (int)work, us, bytes / (us * 1e3));
}

template <int UNROLL, int LDS_KB, bool B, int NT = 0>
static void run(const char* name, const uint8_t* d, uint64_t bytes, uint32_t* out, int blocks, int threads) {
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  for (int w = 0; w < 3; ++w) hipLaunchKernelGGL((probe<UNROLL, LDS_KB, B, NT>), dim3(blocks), dim3(threads), 0, 0, d, bytes, 1200, out);
  CHECK(hipDeviceSynchronize());
  const int iters = 20;
  CHECK(hipEventRecord(e0, 0));
  for (int w = 0; w < iters; ++w) hipLaunchKernelGGL((probe<UNROLL, LDS_KB, B, NT>), dim3(blocks), dim3(threads), 0, 0, d, bytes, 1200, out);
  CHECK(hipEventRecord(e1, 0));
  CHECK(hipEventSynchronize(e1));
  float ms = 0;
  CHECK(hipEventElapsedTime(&ms, e0, e1));
  const double us = ms * 1000.0 / iters;
  printf("%-46s blocks=%5d threads=%4d  %8.1f us  %7.1f GB/s\n", name, blocks, threads, us, bytes / (us * 1e3));
}

int main() {
  int cus = 0;
  CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  const uint64_t bytes = 1200ull << 20;  // 1M x 1200 B
  uint8_t* d;
  uint32_t* out;
  CHECK(hipMalloc(&d, bytes));
  CHECK(hipMalloc(&out, 64 << 20));
  CHECK(hipMemset(d, 0x5a, bytes));
  printf("CUs=%d, buffer %.2f GB\n", cus, bytes / 1e9);
  if (0) run<8, 144, false>("A contiguous, 1x1024/CU, LDS 144K, unroll 8", d, bytes, out, cus, 1024);
  run<16, 144, false>("A contiguous, 1x1024/CU, LDS 144K, unroll 16", d, bytes, out, cus, 1024);
  run<8, 0, false>("A contiguous, 2x1024/CU, unroll 8", d, bytes, out, 2 * cus, 1024);
  run<8, 0, false>("A contiguous, 8x256/CU, unroll 8", d, bytes, out, 8 * cus, 256);
  run<4, 0, false>("A contiguous, 8x256/CU, unroll 4", d, bytes, out, 8 * cus, 256);
  run<8, 0, false>("A contiguous, 4096 blocks x256, unroll 8", d, bytes, out, 4096, 256);
  run<10, 144, true>("B crc-shape, 1x1024/CU, LDS 144K, unroll 10", d, bytes, out, cus, 1024);
  run<5, 144, true>("B crc-shape, 1x1024/CU, LDS 144K, unroll 5", d, bytes, out, cus, 1024);
  run<10, 0, true>("B crc-shape, 2x1024/CU, unroll 10", d, bytes, out, 2 * cus, 1024);
  run<10, 0, true>("B crc-shape, 8x256/CU, unroll 10", d, bytes, out, 8 * cus, 256);
  run<8, 144, false, 1>("A nt, 1x1024/CU, LDS 144K, unroll 8", d, bytes, out, cus, 1024);
  run<4, 0, false, 1>("A nt, 8x256/CU, unroll 4", d, bytes, out, 8 * cus, 256);
  run<10, 144, true, 1>("B nt crc-shape, 1x1024/CU, LDS 144K, unroll 10", d, bytes, out, cus, 1024);
  for (int work : {0, 16, 32}) {
    if (work) continue;
    run_deep<10, 1>("16 waves/CU (1x1024, 144K LDS)", d, bytes, out, cus, work);
    run_deep<10, 1, false, 4>("32 waves/CU (2x1024, 4K LDS)", d, bytes, out, 2 * cus, work);
    run_deep<10, 1, false, 4>("32 waves/CU (8x256, 4K LDS)", d, bytes, out, 8 * cus, work, 256);
    run_deep<5, 1, false, 4>("32 waves/CU NS=5 ring (8x256)", d, bytes, out, 8 * cus, work, 256);
    run_deep<10, 1, false, 4>("8 waves/CU (1x512)", d, bytes, out, cus, work, 512);
  }

  for (int work : {0, 16, 32}) {
    run_dma<8>("DMA ring 8 x 1KiB/wave", d, bytes, out, cus, work);
    run_dma<2>("DMA ring 2 x 1KiB/wave", d, bytes, out, cus, work);
    run_dma1<140>("DMA single 1KiB/wave + 140K pad", d, bytes, out, cus, work);
  }
  return 0;
}
