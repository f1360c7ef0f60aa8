// Probe (tooling, round 6): do the ragged load shapes of tools/dma_shape keep their order once
// each wave also does the CRC's table lookups on what it loads?  VERDICT r5 item 1 asks for
// 4-packet rounds of 16 lanes per packet (one 1-KiB LDS-DMA per compute slot: dma_shape's
// fastest shape at 1392 B) for long datagrams.  16 lanes per packet make each lane's Horner
// step M32^64 instead of M32^32: either the main table applied twice (K = 2: 32 lookups per
// lane per KiB, no new table) or an M32^64 table of its own (K = 1, 32 KiB more LDS that the
// ragged kernel does not have).  The product's 8-lane pair shape does 16 lookups per lane per
// KiB.  Same walk as dma_shape (rounds of P back-to-back packets of L bytes from the packet
// ends backwards, a ring D slots deep, I DMA instructions per slot); per landed 16 B the lane
// does K passes of the product's lookup (4 v_perm + 4 conflict-free ds_read_b32 from the
// replicated 64-KiB block + 2 v_bitop3 per word; ONE asm statement per pass with one
// lgkmcnt(0), as horner_step_and_read).  LDS padded to the jobs kernel's 159 KiB.
//   hipcc --offload-arch=gfx950 -O3 -std=c++20 -o tools/shape_arith tools/shape_arith.hip
//   tools/shape_arith [L=1392] [packets=1605632]
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <vector>

typedef __attribute__((address_space(3))) void LdsVoid;
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

constexpr int kWaves = 16;
constexpr int kLdsBytes = 159 * 1024;
constexpr int kTableBytes = 64 * 1024;  // the replicated block at LDS address 0

template <int N>
__device__ __forceinline__ u32x4 read_landed(uint32_t addr) {
  u32x4 v;
  asm volatile("s_waitcnt vmcnt(%1)\n\tds_read_b128 %0, %2\n\ts_waitcnt lgkmcnt(0)"
               : "=v"(v)
               : "i"(N), "v"(addr)
               : "memory");
  return v;
}

__device__ __forceinline__ u32x4 read_lds(uint32_t addr) {
  u32x4 v;
  asm volatile("ds_read_b128 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(addr) : "memory");
  return v;
}

// h_j <- T(h_j) ^ w_j for the 4 words (T: 4 lookups in the replicated block, lane l reading
// copy l & 7 of table j ^ ((l >> 3) & 3): one v_perm per address, conflict-free).
struct Lk {
  uint32_t lp, sel[4];
};
__device__ __forceinline__ void lookup_pass(const Lk& lk, u32x4& h, u32x4 w) {
  uint32_t a[16];
  const uint32_t hs[4] = {h.x, h.y, h.z, h.w};
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int t = 0; t < 4; ++t) a[4 * j + t] = __builtin_amdgcn_perm(hs[j], lk.lp, lk.sel[t]);
  uint32_t o0, o1, o2, o3;
  asm volatile(
      "ds_read_b32 %4, %4\n\tds_read_b32 %5, %5\n\tds_read_b32 %6, %6\n\tds_read_b32 %7, %7\n\t"
      "ds_read_b32 %8, %8\n\tds_read_b32 %9, %9\n\tds_read_b32 %10, %10\n\tds_read_b32 %11, %11\n\t"
      "ds_read_b32 %12, %12\n\tds_read_b32 %13, %13\n\tds_read_b32 %14, %14\n\tds_read_b32 %15, %15\n\t"
      "ds_read_b32 %16, %16\n\tds_read_b32 %17, %17\n\tds_read_b32 %18, %18\n\tds_read_b32 %19, %19\n\t"
      "s_waitcnt lgkmcnt(0)\n\t"
      "v_bitop3_b32 %4, %4, %5, %6 bitop3:0x96\n\t"
      "v_bitop3_b32 %0, %4, %7, %20 bitop3:0x96\n\t"
      "v_bitop3_b32 %8, %8, %9, %10 bitop3:0x96\n\t"
      "v_bitop3_b32 %1, %8, %11, %21 bitop3:0x96\n\t"
      "v_bitop3_b32 %12, %12, %13, %14 bitop3:0x96\n\t"
      "v_bitop3_b32 %2, %12, %15, %22 bitop3:0x96\n\t"
      "v_bitop3_b32 %16, %16, %17, %18 bitop3:0x96\n\t"
      "v_bitop3_b32 %3, %16, %19, %23 bitop3:0x96"
      : "=&v"(o0), "=&v"(o1), "=&v"(o2), "=&v"(o3), "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]), "+v"(a[4]),
        "+v"(a[5]), "+v"(a[6]), "+v"(a[7]), "+v"(a[8]), "+v"(a[9]), "+v"(a[10]), "+v"(a[11]), "+v"(a[12]),
        "+v"(a[13]), "+v"(a[14]), "+v"(a[15])
      : "v"(w.x), "v"(w.y), "v"(w.z), "v"(w.w)
      : "memory");
  h = u32x4{o0, o1, o2, o3};
}

// P packets per round, PIECE bytes per packet per slot, I DMA instructions per slot, ring of
// D slots, K lookup passes per landed 16 B.
template <int P, int PIECE, int I, int D, int K>
__global__ __launch_bounds__(1024) void arith_kernel(const uint8_t* base, uint32_t L, uint64_t rounds, uint32_t* out) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[kLdsBytes];
  constexpr int kLanesPerPkt = PIECE / 16;
  static_assert(P * PIECE == 1024 * I, "a slot is I KiB");
  static_assert(kTableBytes + D * I * kWaves * 1024 <= kLdsBytes, "LDS");
  const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  for (uint32_t x = threadIdx.x; x < kTableBytes / 4; x += 1024) reinterpret_cast<uint32_t*>(lds)[x] = x * 2654435761u;
  __syncthreads();
  if ((uint32_t)(uintptr_t)(LdsVoid*)lds != 0) __builtin_trap();  // the lookups use raw addresses
  Lk lk;
  {
    const uint32_t oct = (lane >> 3) & 3u, copy = lane & 7u;
    lk.lp = 0;
    for (uint32_t j = 0; j < 4; ++j) {
      const uint32_t t = j ^ oct;
      lk.lp |= (copy * 4u + 32u * t) << (8u * j);
      lk.sel[j] = 0x0C0C0000u | ((4u + t) << 8) | j;
    }
  }
  const uint32_t ns = (L + PIECE - 1) / PIECE;
  const uint64_t gw = (uint64_t)blockIdx.x * kWaves + wv, nw = (uint64_t)gridDim.x * kWaves;
  const uint64_t my_rounds = gw < rounds ? (rounds - gw + nw - 1) / nw : 0;
  const uint64_t q_end = my_rounds * ns;
  if (my_rounds == 0) return;
  auto ring_addr = [&](uint32_t pos, uint32_t i) -> uint32_t {
    return (uint32_t)(kTableBytes + ((pos * I + i) * kWaves + wv) * 1024);
  };
  const uint64_t last_round = my_rounds - 1;
  auto src = [&](uint64_t j, uint32_t s, uint32_t i) -> const uint8_t* {
    const uint64_t r = gw + j * nw;
    const uint32_t t = ns - 1 - s;
    const uint32_t pkt = i * (64 / kLanesPerPkt) + lane / kLanesPerPkt, k = lane % kLanesPerPkt;
    const uint8_t* end = base + (r * P + pkt + 1) * (uint64_t)L;
    return end - (uint64_t)PIECE * (t + 1) + 16 * k;
  };
  uint64_t dj = 0;
  uint32_t dsl = 0;
  auto advance = [&]() {
    if (dj == last_round && dsl == ns - 1) return;
    if (++dsl == ns) {
      dsl = 0;
      ++dj;
    }
  };
#pragma unroll
  for (int d = 0; d < D; ++d) {
#pragma unroll
    for (int i = 0; i < I; ++i)
      __builtin_amdgcn_global_load_lds((const void*)src(dj, dsl, i), (LdsVoid*)(lds + ring_addr(d, i)), 16, 0, 0);
    advance();
  }
  u32x4 h = {lane, 0, 0, 0};
  uint32_t pos = 0;
  for (uint64_t q = 0; q < q_end; ++q) {
    u32x4 v[I];
    v[0] = read_landed<(D - 1) * I>(ring_addr(pos, 0) + 16 * lane);
#pragma unroll
    for (int i = 1; i < I; ++i) v[i] = read_lds(ring_addr(pos, i) + 16 * lane);
#pragma unroll
    for (int i = 0; i < I; ++i)
      __builtin_amdgcn_global_load_lds((const void*)src(dj, dsl, i), (LdsVoid*)(lds + ring_addr(pos, i)), 16, 0, 0);
    advance();
    pos = pos + 1 == D ? 0 : pos + 1;
#pragma unroll
    for (int i = 0; i < I; ++i) {
#pragma unroll
      for (int k = 0; k < K; ++k) lookup_pass(lk, h, k == K - 1 ? v[i] : u32x4{0, 0, 0, 0});
    }
  }
  __builtin_amdgcn_s_waitcnt(0);
  out[(blockIdx.x * 1024 + threadIdx.x)] = h.x ^ h.y ^ h.z ^ h.w;
}

struct Shape {
  const char* name;
  int P;
  void (*launch)(int grid, const uint8_t*, uint32_t, uint64_t, uint32_t*);
};

template <int P, int PIECE, int I, int D, int K>
void launch_shape(int grid, const uint8_t* b, uint32_t L, uint64_t rounds, uint32_t* out) {
  hipLaunchKernelGGL((arith_kernel<P, PIECE, I, D, K>), dim3(grid), dim3(1024), 0, 0, b, L, rounds, out);
}

#define CHECK(x)                                                             \
  do {                                                                       \
    hipError_t e_ = (x);                                                     \
    if (e_ != hipSuccess) {                                                  \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                \
      return 2;                                                              \
    }                                                                        \
  } while (0)

int main(int argc, char** argv) {
  const uint32_t L = argc > 1 ? (uint32_t)atoi(argv[1]) : 1392;
  uint64_t n = argc > 2 ? strtoull(argv[2], nullptr, 10) : 1605632;
  n -= n % 16;
  if (L < 16 || L > 65536) return 1;
  // name: P x PIECE x I, ring depth, lookup passes per 16 B (16 lookups per lane per pass)
  const Shape shapes[] = {
      {"8x256x2 d2 K1 (product pairs)", 8, launch_shape<8, 256, 2, 2, 1>},
      {"8x256x2 d2 K0 (loads only)", 8, launch_shape<8, 256, 2, 2, 0>},
      {"4x256x1 d2 K0 (loads only)", 4, launch_shape<4, 256, 1, 2, 0>},
      {"4x256x1 d2 K1 (M32^64 table)", 4, launch_shape<4, 256, 1, 2, 1>},
      {"4x256x1 d2 K2 (M32^32 twice)", 4, launch_shape<4, 256, 1, 2, 2>},
      {"4x256x1 d3 K2", 4, launch_shape<4, 256, 1, 3, 2>},
      {"4x256x1 d4 K2", 4, launch_shape<4, 256, 1, 4, 2>},
      {"4x256x1 d4 K1", 4, launch_shape<4, 256, 1, 4, 1>},
      {"8x256x2 d1 K1", 8, launch_shape<8, 256, 2, 1, 1>},
  };
  const int ns = sizeof(shapes) / sizeof(shapes[0]);
  hipDeviceProp_t prop;
  CHECK(hipGetDeviceProperties(&prop, 0));
  const int grid = prop.multiProcessorCount;
  const uint64_t bytes = n * L;
  uint8_t* buf = nullptr;
  uint32_t* out = nullptr;
  CHECK(hipMalloc(&buf, bytes + 8192));
  CHECK(hipMalloc(&out, (size_t)grid * 1024 * 4));
  CHECK(hipMemset(buf, 0x5a, bytes + 8192));
  const uint8_t* base = buf + 4096;  // a piece reaches at most PIECE - 16 B before its packet
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  printf("L=%u packets=%llu bytes=%llu grid=%d\n", L, (unsigned long long)n, (unsigned long long)bytes, grid);
  fflush(stdout);
  for (int w = 0; w < 80; ++w) shapes[w % ns].launch(grid, base, L, n / shapes[w % ns].P, out);
  CHECK(hipGetLastError());
  CHECK(hipDeviceSynchronize());
  std::vector<std::vector<float>> us(ns);
  const int kBlocks = 8, kLaunches = 20;
  for (int blk = 0; blk < kBlocks; ++blk)
    for (int j = 0; j < ns; ++j) {
      const int s = blk % 2 ? ns - 1 - j : j;
      shapes[s].launch(grid, base, L, n / shapes[s].P, out);
      CHECK(hipEventRecord(e0, 0));
      for (int it = 0; it < kLaunches; ++it) shapes[s].launch(grid, base, L, n / shapes[s].P, out);
      CHECK(hipEventRecord(e1, 0));
      CHECK(hipEventSynchronize(e1));
      float ms = 0;
      CHECK(hipEventElapsedTime(&ms, e0, e1));
      us[s].push_back(1000.f * ms / kLaunches);
    }
  for (int s = 0; s < ns; ++s) {
    std::vector<float> v = us[s];
    std::sort(v.begin(), v.end());
    const float med = 0.5f * (v[kBlocks / 2 - 1] + v[kBlocks / 2]);
    printf("%-32s median %8.1f us  (%7.1f-%7.1f)  %6.0f GB/s  %.3f of 8 TB/s\n", shapes[s].name, med, v.front(),
           v.back(), bytes / (med * 1e-6) / 1e9, bytes / (med * 1e-6) / 8e12);
  }
  CHECK(hipFree(buf));
  CHECK(hipFree(out));
  return 0;
}
