// Probe (tooling): does the SHAPE of a ragged kernel's LDS-DMA stream change what it
// streams?  No CRC arithmetic: each wave walks rounds of P back-to-back packets of L bytes
// from the packet ends backwards, one slot per step, exactly as the ragged kernels load
// (lane k of a packet's group reads 16 B at end - PIECE*(t+1) + 16k into an LDS ring,
// D slots deep, I DMA instructions per slot), reads its own 16 B of every landed slot back
// and XORs it in.  Shapes:
//   8x128x1 d3   the 8-lane kernel (8 packets per instruction, 128-B pieces, ring of 3)
//   16x64x1 d3   the 16-packet kernel (16 packets per instruction, 64-B pieces)
//   16x128x2 d2  16 packets per round loaded as two 8x128 instructions, ring of 2
//   16x128x2 d3  the same, ring of 3
//   8x128x1 d2   the 8-lane shape with a ring of 2
//   4x256x1 d2/3 16 lanes per packet (256-B pieces of 4 packets)
//   2x512x1 d2   32 lanes per packet
//   16x128x2 d1  two 8x128 instructions per slot, one slot in flight
//   8x128 regs   the 8-lane shape loaded into a register ring (3 or 6 deep; nt: non-temporal)
//   8x256x2 d2/3 8 packets x 256 B per 2-KiB slot as two 4 x 256-B instructions (the round-5 plan)
//   4x256x1 d4, 8x256x2 d1, 4x512x2 d2, 2x512x1 d4: the same bytes in flight with other packet counts
//   ... nt: the LDS-DMA shapes with the non-temporal hint (round 6)
// Workgroups of 1024 threads, one per CU (the LDS is padded to the kernels' 150 KiB), a
// persistent grid over static rounds.  Alternating blocks of 20 launches per shape after a
// warm-up; prints us per launch and GB/s.  Addresses stay inside the buffer: the packets
// start 4 KiB into the allocation and a chunk never reaches more than 128 B before a packet.
//   hipcc --offload-arch=gfx950 -O3 -o tools/dma_shape tools/dma_shape.hip
//   tools/dma_shape [L=1392] [packets=1605632] [base_offset=0] [align=1: piece starts rounded down to this]
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <vector>

typedef __attribute__((address_space(3))) void LdsVoid;
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

constexpr int kWaves = 16;
constexpr int kLdsBytes = 150 * 1024;

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

// P packets per round, PIECE bytes per packet per slot, I instructions per slot, ring of D.
template <int P, int PIECE, int I, int D, int kAux = 0>
__global__ __launch_bounds__(1024) void shape_kernel(const uint8_t* base, uint32_t L, uint64_t rounds,
                                                     uint64_t amask, uint32_t* out) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[kLdsBytes];
  constexpr int kLanesPerPkt = PIECE / 16;
  static_assert(P * PIECE == 1024 * I, "a slot is I KiB");
  const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const uint32_t ns = (L + PIECE - 1) / PIECE;
  const uint64_t gw = (uint64_t)blockIdx.x * kWaves + wv, nw = (uint64_t)gridDim.x * kWaves;
  const uint64_t my_rounds = gw < rounds ? (rounds - gw + nw - 1) / nw : 0;
  const uint64_t q_end = my_rounds * ns;
  if (my_rounds == 0) return;
  // ring[pos][i][wave][64] of u32x4
  auto ring_addr = [&](uint32_t pos, uint32_t i) -> uint32_t {
    return (uint32_t)(((pos * I + i) * kWaves + wv) * 1024);
  };
  // DMA cursor: round j of this wave (round gw + j*nw), slot s; past the last slot of the
  // last round it stays on that slot (re-reads keep vmcnt exact).
  const uint64_t last_round = my_rounds - 1;
  auto src = [&](uint64_t j, uint32_t s, uint32_t i) -> const uint8_t* {
    const uint64_t r = gw + j * nw;
    const uint32_t t = ns - 1 - s;
    const uint32_t pkt = i * (64 / kLanesPerPkt) + lane / kLanesPerPkt, k = lane % kLanesPerPkt;
    const uint8_t* end = base + (r * P + pkt + 1) * (uint64_t)L;
    return (const uint8_t*)(((uint64_t)(end - (uint64_t)PIECE * (t + 1)) & amask) + 16 * k);
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
  u32x4 acc = {0, 0, 0, 0};
#pragma unroll
  for (int d = 0; d < D; ++d) {
#pragma unroll
    for (int i = 0; i < I; ++i)
      __builtin_amdgcn_global_load_lds((const void*)src(dj, dsl, i), (LdsVoid*)(lds + ring_addr(d, i)), 16, 0, kAux);
    advance();
  }
  uint32_t pos = 0;
  for (uint64_t q = 0; q < q_end; ++q) {
    acc ^= read_landed<(D - 1) * I>(ring_addr(pos, 0) + 16 * lane);  // both instructions of the slot
#pragma unroll
    for (int i = 1; i < I; ++i) acc ^= read_lds(ring_addr(pos, i) + 16 * lane);
#pragma unroll
    for (int i = 0; i < I; ++i)
      __builtin_amdgcn_global_load_lds((const void*)src(dj, dsl, i), (LdsVoid*)(lds + ring_addr(pos, i)), 16, 0, kAux);
    advance();
    pos = pos + 1 == D ? 0 : pos + 1;
  }
  __builtin_amdgcn_s_waitcnt(0);
  out[(blockIdx.x * 1024 + threadIdx.x)] = acc.x ^ acc.y ^ acc.z ^ acc.w;
}

// The same walk with the pieces loaded into a register ring (global_load_dwordx4, D slots
// deep, optionally non-temporal) instead of LDS-DMA: the G1 kernel's load form.
template <int P, int PIECE, int D, bool kNT>
__global__ __launch_bounds__(1024) void shape_regs_kernel(const uint8_t* base, uint32_t L, uint64_t rounds,
                                                          uint64_t amask, uint32_t* out) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[kLdsBytes];  // same occupancy as the DMA form
  constexpr int kLanesPerPkt = PIECE / 16;
  static_assert(P * PIECE == 1024, "one instruction per slot");
  const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
  const uint32_t ns = (L + PIECE - 1) / PIECE;
  const uint64_t gw = (uint64_t)blockIdx.x * kWaves + wv, nw = (uint64_t)gridDim.x * kWaves;
  const uint64_t my_rounds = gw < rounds ? (rounds - gw + nw - 1) / nw : 0;
  if (my_rounds == 0) return;
  const uint64_t q_end = my_rounds * ns;
  const uint64_t last_round = my_rounds - 1;
  const uint32_t pkt = lane / kLanesPerPkt, k = lane % kLanesPerPkt;
  auto src = [&](uint64_t j, uint32_t s) -> const u32x4* {
    const uint64_t r = gw + j * nw;
    const uint8_t* end = base + (r * P + pkt + 1) * (uint64_t)L;
    return (const u32x4*)((((uint64_t)(end - (uint64_t)PIECE * (ns - s))) & amask) + 16 * k);
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
  u32x4 ring[D];
  u32x4 acc = {0, 0, 0, 0};
#pragma unroll
  for (int d = 0; d < D; ++d) {
    ring[d] = kNT ? __builtin_nontemporal_load(src(dj, dsl)) : *src(dj, dsl);
    advance();
    __builtin_amdgcn_sched_barrier(0);
  }
  for (uint64_t q = 0; q + D <= q_end + D - 1; q += D) {
#pragma unroll
    for (int d = 0; d < D; ++d) {
      acc ^= ring[d];
      ring[d] = kNT ? __builtin_nontemporal_load(src(dj, dsl)) : *src(dj, dsl);
      advance();
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  if (lane == 0) lds[wv] = (uint8_t)acc.x;
  out[(blockIdx.x * 1024 + threadIdx.x)] = acc.x ^ acc.y ^ acc.z ^ acc.w;
}

struct Shape {
  const char* name;
  int P;
  void (*launch)(int grid, const uint8_t*, uint32_t, uint64_t, uint64_t, uint32_t*);
};

template <int P, int PIECE, int D, bool kNT>
void launch_regs(int grid, const uint8_t* b, uint32_t L, uint64_t rounds, uint64_t amask, uint32_t* out) {
  hipLaunchKernelGGL((shape_regs_kernel<P, PIECE, D, kNT>), dim3(grid), dim3(1024), 0, 0, b, L, rounds, amask, out);
}

template <int P, int PIECE, int I, int D, int kAux = 0>
void launch_shape(int grid, const uint8_t* b, uint32_t L, uint64_t rounds, uint64_t amask, uint32_t* out) {
  hipLaunchKernelGGL((shape_kernel<P, PIECE, I, D, kAux>), dim3(grid), dim3(1024), 0, 0, b, L, rounds, amask, out);
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
  const uint32_t off = argc > 3 ? (uint32_t)atoi(argv[3]) : 0;
  // align=A (a power of two): every piece's start rounded down to an A-byte boundary (16: the
  // lane loads 16-B aligned; 128 with 128-B pieces: whole lines, the G1 kernel's loads)
  const uint64_t align = argc > 4 ? (uint64_t)atoi(argv[4]) : 1;
  if (align == 0 || (align & (align - 1)) || align > 1024) return 1;
  const uint64_t amask = ~(align - 1);
  n -= n % 16;  // whole rounds for every shape
  if (L < 16 || L > 65536 || off > 64) return 1;
  const Shape shapes[] = {
      {"8x128x1 d3", 8, launch_shape<8, 128, 1, 3>},   {"16x64x1 d3", 16, launch_shape<16, 64, 1, 3>},
      {"16x128x2 d2", 16, launch_shape<16, 128, 2, 2>}, {"16x128x2 d3", 16, launch_shape<16, 128, 2, 3>},
      {"8x128x1 d2", 8, launch_shape<8, 128, 1, 2>},   {"4x256x1 d2", 4, launch_shape<4, 256, 1, 2>},
      {"4x256x1 d3", 4, launch_shape<4, 256, 1, 3>},   {"2x512x1 d2", 2, launch_shape<2, 512, 1, 2>},
      {"16x128x2 d1", 16, launch_shape<16, 128, 2, 1>},
      {"8x256x2 d2", 8, launch_shape<8, 256, 2, 2>},   {"8x256x2 d3", 8, launch_shape<8, 256, 2, 3>},
      {"8x128 regs d3", 8, launch_regs<8, 128, 3, false>}, {"8x128 regs d6", 8, launch_regs<8, 128, 6, false>},
      {"8x128 regsnt d6", 8, launch_regs<8, 128, 6, true>},
      // round-5 additions: in-flight bytes vs packets per wave
      {"4x256x1 d4", 4, launch_shape<4, 256, 1, 4>},   {"8x256x2 d1", 8, launch_shape<8, 256, 2, 1>},
      {"4x512x2 d2", 4, launch_shape<4, 512, 2, 2>},   {"2x512x1 d4", 2, launch_shape<2, 512, 1, 4>},
      // round-6 additions: the LDS-DMA shapes with the non-temporal hint (aux 2, as the uniform DMA kernels)
      {"8x256x2 d2 nt", 8, launch_shape<8, 256, 2, 2, 2>}, {"8x128x1 d3 nt", 8, launch_shape<8, 128, 1, 3, 2>},
      {"4x256x1 d2 nt", 4, launch_shape<4, 256, 1, 2, 2>}, {"8x256x2 d1 nt", 8, launch_shape<8, 256, 2, 1, 2>},
      {"8x128x1 d6 nt", 8, launch_shape<8, 128, 1, 6, 2>}, {"8x128x1 d4 nt", 8, launch_shape<8, 128, 1, 4, 2>},
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
  const uint8_t* base = buf + 4096 + off;  // pieces rounded down by up to 1023 B stay inside the allocation
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  printf("L=%u packets=%llu bytes=%llu base_offset=%u align=%llu grid=%d\n", L, (unsigned long long)n,
         (unsigned long long)bytes, off, (unsigned long long)align, grid);
  // warm-up through the power-management transient
  for (int w = 0; w < 60; ++w) shapes[w % ns].launch(grid, base, L, n / shapes[w % ns].P, amask, out);
  CHECK(hipGetLastError());
  CHECK(hipDeviceSynchronize());
  std::vector<std::vector<float>> us(ns);
  const int kBlocks = 6, kLaunches = 20;
  for (int blk = 0; blk < kBlocks; ++blk)
    for (int j = 0; j < ns; ++j) {
      const int s = blk % 2 ? ns - 1 - j : j;
      shapes[s].launch(grid, base, L, n / shapes[s].P, amask, out);
      CHECK(hipEventRecord(e0, 0));
      for (int it = 0; it < kLaunches; ++it) shapes[s].launch(grid, base, L, n / shapes[s].P, amask, out);
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
    printf("%-12s median %8.1f us  (%7.1f-%7.1f)  %6.0f GB/s\n", shapes[s].name, med, v.front(), v.back(),
           bytes / (med * 1e-6) / 1e9);
  }
  CHECK(hipFree(buf));
  CHECK(hipFree(out));
  return 0;
}
