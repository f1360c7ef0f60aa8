// LDS-DMA streaming probe (tooling, not product): does the ACCESS PATTERN of the
// CRC kernel's DMA ring limit its bandwidth?  Same ring as crc32_uniform_dma_kernel
// (5 x 1 KiB per wave, 16 waves/CU, 80 KiB of other LDS), same asm waits.
//   pattern 0: global streaming, wave's slot t = 1 KiB piece (t * nwaves + wave)
//   pattern 1: CRC kernel shape, 8 packets x 128 B at packet offset 128 s - 80 (1200-B packets)
//   pattern 2: CRC shape, 16-B aligned within the packet (offset 128 s)
//   pattern 3: block-contiguous: round = 8 packets = 9600 B, slot s = bytes [1024 s, +1024)
// work = 0: XOR only; work = 1: 16 table lookups per slot (the kernel's per-slot LDS load).
//   hipcc --offload-arch=gfx950 -O3 -o tools/dma_probe tools/dma_probe.hip
#include <hip/hip_runtime.h>
#include "../rusty_enet_amd/csrc/crc32_layout.hpp"
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void LdsVoid;
#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

constexpr int NS = 10;

template <int R>
__device__ __forceinline__ u32x4 read_slot(uint32_t a) {
  u32x4 v;
  asm volatile("s_waitcnt vmcnt(%2)\n\tds_read_b128 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(a), "i"(R - 1) : "memory");
  return v;
}

template <int PAT, int WORK, int NT, int R = 5>
__global__ __launch_bounds__(1024) void probe(const uint8_t* __restrict__ buf, uint64_t npk, uint32_t* __restrict__ out) {
  constexpr int kTab = R <= 5 ? 20480 : (R == 6 ? 16384 : (R == 7 ? 12288 : 4096));
  __shared__ __attribute__((aligned(16))) uint32_t tab[kTab];
  __shared__ __attribute__((aligned(16))) u32x4 ring[R][16][64];
  for (int i = threadIdx.x; i < kTab; i += 1024) tab[i] = i * 2654435761u;
  __syncthreads();
  const uint32_t lane = threadIdx.x & 63, wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const enet_crc::Lookup lk = enet_crc::make_lookup(lane);
  const uint32_t g = lane / 8, k = lane % 8;
  const uint64_t wave = (uint64_t)blockIdx.x * 16 + wv, nwaves = (uint64_t)gridDim.x * 16;
  const uint64_t nrounds_total = npk / 8;
  const uint64_t nr = wave < nrounds_total ? (nrounds_total - wave + nwaves - 1) / nwaves : 0;
  const uint64_t base = (uint64_t)(uintptr_t)buf;
  auto src = [&](uint64_t r, int s) -> uint64_t {
    const uint64_t rr = wave + (r < nr ? r : nr - 1) * nwaves;  // global round index
    if (PAT == 0) return base + ((uint64_t)(rr * NS + s) % (npk * 1200 / 1024)) * 1024 + lane * 16;
    if (PAT == 3) return base + rr * 9600 + (uint64_t)s * 1024 + lane * 16;
    // 1280-B packets (10 whole lines): 6 = 8 packets x one aligned line per slot (the
    // 64-KiB kernel's shape), 8 = the same 10 KiB read as contiguous KiB.
    if (PAT == 6) return base + (rr * 8 + g) * 1280 + (uint64_t)s * 128 + 16 * k;
    if (PAT == 8) return base + rr * 10240 + (uint64_t)s * 1024 + lane * 16;
    // 1200-B packets with every line of the round's 75 read once, whole: group g takes
    // lines [1200 g / 128, 1200 (g + 1) / 128) of the 9600-B round (9 or 10 lines; a 10th
    // slot of a 9-line group re-reads the buffer's first line, L2-resident): the shape a
    // line-split DMA ring with the shared boundary line handed between groups would have.
    if (PAT == 9) {
      const uint32_t l0 = (1200u * g) / 128u, l1 = (1200u * (g + 1)) / 128u, line = l0 + (uint32_t)s;
      return line >= l1 ? base + 16 * k : base + rr * 9600 + (uint64_t)line * 128 + 16 * k;
    }
    if (PAT == 5) {  // 16 lanes per packet: slots 0-4 packets 0-3 of the round, slots 5-9 packets 4-7
      const uint64_t pk = rr * 8 + (s / 5) * 4 + lane / 16;
      int64_t off = -80 + 256 * (s % 5) + 16 * (int)(lane % 16);
      if (off < 0 && pk == 0) off = 0;
      if (off + 16 > 1200) off = 1200 - 16;
      return base + pk * 1200 + off;
    }
    const uint64_t pb = base + (rr * 8 + g) * 1200;
    int64_t off = (PAT == 1 || PAT == 4 ? -80 : 0) + 128 * s + 16 * (int)(PAT == 4 ? 7 - k : k);
    if (off < 0 && rr * 8 + g == 0) off = 0;
    if (off + 16 > 1200) off = 1200 - 16;
    return pb + off;
  };
  auto dma = [&](uint64_t a, uint32_t q) {
    __builtin_amdgcn_global_load_lds((const void*)a, (LdsVoid*)&ring[q][wv][0], 16, 0, NT ? 2 : 0);
  };
  if (nr == 0) return;
  const uint64_t t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  for (int f = 0; f < R; ++f) dma(src(f / NS, f % NS), f);
  const uint32_t ring0 = (uint32_t)(uintptr_t)(LdsVoid*)&ring[0][wv][0];
  uint32_t q = 0, h0 = lane, h1 = lane * 3, h2 = lane * 5, h3 = lane * 7;
  for (uint64_t r = 0; r < nr; ++r) {
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      const u32x4 v = read_slot<R>(ring0 + q * 16384u + lane * 16u);
      const int f = s + R;
      dma(src(r + f / NS, f % NS), q);
      q = q + 1 == R ? 0 : q + 1;
      if (WORK == 2) {  // the kernel's slot work: 16 conflict-free lookups (crc32_layout.hpp)
        auto step = [&](uint32_t h, uint32_t w) {
          return tab[enet_crc::lookup_addr(h, lk.lp, lk, 0) / 4] ^ tab[enet_crc::lookup_addr(h, lk.lp, lk, 1) / 4] ^
                 tab[enet_crc::lookup_addr(h, lk.lp, lk, 2) / 4] ^ tab[enet_crc::lookup_addr(h, lk.lp, lk, 3) / 4] ^ w;
        };
        h0 = step(h0, v.x); h1 = step(h1, v.y); h2 = step(h2, v.z); h3 = step(h3, v.w);
      } else if (WORK) {
        auto step = [&](uint32_t h, uint32_t w) {
          return tab[h & 0xff] ^ tab[256 + ((h >> 8) & 0xff)] ^ tab[512 + ((h >> 16) & 0xff)] ^ tab[768 + (h >> 24)] ^ w;
        };
        h0 = step(h0, v.x); h1 = step(h1, v.y); h2 = step(h2, v.z); h3 = step(h3, v.w);
      } else {
        h0 ^= v.x; h1 ^= v.y; h2 ^= v.z; h3 ^= v.w;
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  __builtin_amdgcn_s_waitcnt(0);
  out[blockIdx.x * 1024 + threadIdx.x] = h0 ^ h1 ^ h2 ^ h3;
  if (threadIdx.x == 0) {  // diagnostic clock stamps (own buffer region, never read by the kernel)
    const uint64_t t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    reinterpret_cast<unsigned long long*>(out + (8 << 20))[2 * blockIdx.x] = t1 - t0;
    reinterpret_cast<unsigned long long*>(out + (8 << 20))[2 * blockIdx.x + 1] = r1 - r0;
  }
}


// Register-staged variant: global_load_dwordx4 straight into a per-round VGPR ring
// (round r+1's NS chunks load while round r is processed), kernel-like lookups.
typedef uint32_t u32x4a __attribute__((ext_vector_type(4)));
template <int NT>
__global__ __launch_bounds__(1024) void probe_regs(const uint8_t* __restrict__ buf, uint64_t npk, uint32_t* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) uint32_t tab[16384];
  for (int i = threadIdx.x; i < 16384; i += 1024) tab[i] = i * 2654435761u;
  __syncthreads();
  const uint32_t lane = threadIdx.x & 63, wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const enet_crc::Lookup lk = enet_crc::make_lookup(lane);
  const uint32_t g = lane / 8, k = lane % 8;
  const uint64_t wave = (uint64_t)blockIdx.x * 16 + wv, nwaves = (uint64_t)gridDim.x * 16;
  const uint64_t nrounds_total = npk / 8;
  const uint64_t nr = wave < nrounds_total ? (nrounds_total - wave + nwaves - 1) / nwaves : 0;
  const uint64_t base = (uint64_t)(uintptr_t)buf;
  if (nr == 0) return;
  const uint64_t t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  typedef __attribute__((address_space(1))) const u32x4a G4;
  auto src = [&](uint64_t r, int s) -> G4* {
    const uint64_t rr = wave + (r < nr ? r : nr - 1) * nwaves;
    const uint64_t pb = base + (rr * 8 + g) * 1200;
    int64_t off = -80 + 128 * s + 16 * (int)k;
    if (off < 0 && rr * 8 + g == 0) off = 0;
    return (G4*)(pb + off);
  };
  auto ld = [&](G4* a) -> u32x4a {
    return NT ? __builtin_nontemporal_load(a) : *a;
  };
  u32x4a q[NS];
#pragma unroll
  for (int s = 0; s < NS; ++s) { q[s] = ld(src(0, s)); __builtin_amdgcn_sched_barrier(0); }
  uint32_t h0 = lane, h1 = lane * 3, h2 = lane * 5, h3 = lane * 7;
  auto step = [&](uint32_t h, uint32_t w) {
    return tab[enet_crc::lookup_addr(h, lk.lp, lk, 0) / 4] ^ tab[enet_crc::lookup_addr(h, lk.lp, lk, 1) / 4] ^
           tab[enet_crc::lookup_addr(h, lk.lp, lk, 2) / 4] ^ tab[enet_crc::lookup_addr(h, lk.lp, lk, 3) / 4] ^ w;
  };
  for (uint64_t r = 0; r < nr; ++r) {
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      const u32x4a v = q[s];
      h0 = step(h0, v.x); h1 = step(h1, v.y); h2 = step(h2, v.z); h3 = step(h3, v.w);
      __builtin_amdgcn_sched_barrier(0);
      q[s] = ld(src(r + 1, s));
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  out[blockIdx.x * 1024 + threadIdx.x] = h0 ^ h1 ^ h2 ^ h3;
  if (threadIdx.x == 0) {
    const uint64_t t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    reinterpret_cast<unsigned long long*>(out + (8 << 20))[2 * blockIdx.x] = t1 - t0;
    reinterpret_cast<unsigned long long*>(out + (8 << 20))[2 * blockIdx.x + 1] = r1 - r0;
  }
}

// Line-grid register ring (the shape of an absolute-line G1 kernel): round = 8
// consecutive 1200-B packets, group g = packet; slot s of a lane reads the 16-B chunk
// at line (last_line - 128 (NS-1 - s)) + 16 (7 - k); chunks outside the packet read a
// zero chunk instead (no byte outside [S, E) is ever read).  NTM 0: plain loads, 1: all
// nontemporal, 2: nontemporal except the first two and the last slot (the lines a packet
// shares with its neighbours stay cacheable).
__device__ __attribute__((aligned(64))) uint32_t g_probe_zero[16] = {0};
template <int NSL, int NTM>
__global__ __launch_bounds__(1024) void probe_lines(const uint8_t* __restrict__ buf, uint64_t npk, uint32_t* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) uint32_t tab[16384];
  for (int i = threadIdx.x; i < 16384; i += 1024) tab[i] = i * 2654435761u;
  __syncthreads();
  const uint32_t lane = threadIdx.x & 63, wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const enet_crc::Lookup lk = enet_crc::make_lookup(lane);
  const uint32_t g = lane / 8, k = lane % 8;
  const uint64_t wave = (uint64_t)blockIdx.x * 16 + wv, nwaves = (uint64_t)gridDim.x * 16;
  const uint64_t nrounds_total = npk / 8;
  const uint64_t nr = wave < nrounds_total ? (nrounds_total - wave + nwaves - 1) / nwaves : 0;
  const uint64_t base = (uint64_t)(uintptr_t)buf, zero = (uint64_t)(uintptr_t)g_probe_zero;
  if (nr == 0) return;
  const uint64_t t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  typedef __attribute__((address_space(1))) const u32x4a G4;
  auto src = [&](uint64_t r, int s) -> G4* {
    const uint64_t rr = wave + (r < nr ? r : nr - 1) * nwaves;
    const uint64_t S = base + (rr * 8 + g) * 1200, E = S + 1200;
    const uint64_t A = ((E - 1) & ~(uint64_t)127) - 128u * (NSL - 1 - s) + 16u * (7 - k);
    return (G4*)(A < S || A >= E ? zero : A);
  };
  auto ld = [&](G4* a, int s) -> u32x4a {
    const bool nt = NTM == 1 || (NTM == 2 && s >= 2 && s < NSL - 1);
    return nt ? __builtin_nontemporal_load(a) : *a;
  };
  u32x4a q[NSL];
#pragma unroll
  for (int s = 0; s < NSL; ++s) { q[s] = ld(src(0, s), s); __builtin_amdgcn_sched_barrier(0); }
  uint32_t h0 = lane, h1 = lane * 3, h2 = lane * 5, h3 = lane * 7;
  auto step = [&](uint32_t h, uint32_t w) {
    return tab[enet_crc::lookup_addr(h, lk.lp, lk, 0) / 4] ^ tab[enet_crc::lookup_addr(h, lk.lp, lk, 1) / 4] ^
           tab[enet_crc::lookup_addr(h, lk.lp, lk, 2) / 4] ^ tab[enet_crc::lookup_addr(h, lk.lp, lk, 3) / 4] ^ w;
  };
  for (uint64_t r = 0; r < nr; ++r) {
#pragma unroll
    for (int s = 0; s < NSL; ++s) {
      const u32x4a v = q[s];
      h0 = step(h0, v.x); h1 = step(h1, v.y); h2 = step(h2, v.z); h3 = step(h3, v.w);
      __builtin_amdgcn_sched_barrier(0);
      q[s] = ld(src(r + 1, s), s);
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  out[blockIdx.x * 1024 + threadIdx.x] = h0 ^ h1 ^ h2 ^ h3;
  if (threadIdx.x == 0) {
    const uint64_t t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    reinterpret_cast<unsigned long long*>(out + (8 << 20))[2 * blockIdx.x] = t1 - t0;
    reinterpret_cast<unsigned long long*>(out + (8 << 20))[2 * blockIdx.x + 1] = r1 - r0;
  }
}

// End-aligned pieces from line-aligned loads: the 11 loads of a round each read ONE
// whole 128-B line per group (lane k loads the chunk of that line it owns: piece t if
// k >= j, piece t + 1 if k < j, j = (a1 mod 128) / 16), and slot s takes lane k's chunk
// from ring entry s (k >= j) or s + 1 (k < j): 10 pieces, 9 lookup steps, as now, but no
// line is split between two loads.  NTM 2: non-temporal except the two shared lines.
template <int NTM>
__global__ __launch_bounds__(1024) void probe_linesplit(const uint8_t* __restrict__ buf, uint64_t npk, uint32_t* __restrict__ out) {
  constexpr int NSP = 10;
  __shared__ __attribute__((aligned(16))) uint32_t tab[16384];
  for (int i = threadIdx.x; i < 16384; i += 1024) tab[i] = i * 2654435761u;
  __syncthreads();
  const uint32_t lane = threadIdx.x & 63, wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const enet_crc::Lookup lk = enet_crc::make_lookup(lane);
  const uint32_t g = lane / 8, k = lane % 8;
  const uint64_t wave = (uint64_t)blockIdx.x * 16 + wv, nwaves = (uint64_t)gridDim.x * 16;
  const uint64_t nrounds_total = npk / 8;
  const uint64_t nr = wave < nrounds_total ? (nrounds_total - wave + nwaves - 1) / nwaves : 0;
  const uint64_t base = (uint64_t)(uintptr_t)buf, zero = (uint64_t)(uintptr_t)g_probe_zero;
  if (nr == 0) return;
  const uint64_t t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  typedef __attribute__((address_space(1))) const u32x4a G4;
  auto jj = [&](uint64_t r) -> uint32_t {
    const uint64_t rr = wave + (r < nr ? r : nr - 1) * nwaves;
    return (uint32_t)((base + (rr * 8 + g + 1) * 1200) & 127u) >> 4;
  };
  auto src = [&](uint64_t r, int u) -> G4* {  // ring entry u = line-load t = NSP - 1 - u
    const uint64_t rr = wave + (r < nr ? r : nr - 1) * nwaves;
    const uint64_t a1 = base + (rr * 8 + g + 1) * 1200;
    const uint32_t j = (uint32_t)(a1 & 127u) >> 4;
    const int pi = (NSP - 1 - u) + (k < j ? 1 : 0);
    const bool real = pi >= 0 && pi < NSP && !(rr * 8 + g == 0 && pi == NSP - 1);
    return (G4*)(real ? a1 - 128u * (uint64_t)pi - 16u * (k + 1) : zero);
  };
  auto ld = [&](G4* a, int u) -> u32x4a {
    const bool nt = NTM == 1 || (NTM == 2 && u >= 1 && u < NSP);
    return nt ? __builtin_nontemporal_load(a) : *a;
  };
  u32x4a q[NSP + 1];
#pragma unroll
  for (int u = 0; u <= NSP; ++u) { q[u] = ld(src(0, u), u); __builtin_amdgcn_sched_barrier(0); }
  uint32_t h0 = lane, h1 = lane * 3, h2 = lane * 5, h3 = lane * 7;
  auto step = [&](uint32_t h, uint32_t w) {
    return tab[enet_crc::lookup_addr(h, lk.lp, lk, 0) / 4] ^ tab[enet_crc::lookup_addr(h, lk.lp, lk, 1) / 4] ^
           tab[enet_crc::lookup_addr(h, lk.lp, lk, 2) / 4] ^ tab[enet_crc::lookup_addr(h, lk.lp, lk, 3) / 4] ^ w;
  };
  uint32_t j = jj(0);
  for (uint64_t r = 0; r < nr; ++r) {
    const bool lo = k < j;
#pragma unroll
    for (int s = 0; s < NSP; ++s) {
      const u32x4a v = lo ? q[s + 1] : q[s];
      if (s == 0) { h0 = v.x; h1 = v.y; h2 = v.z; h3 = v.w; }
      else { h0 = step(h0, v.x); h1 = step(h1, v.y); h2 = step(h2, v.z); h3 = step(h3, v.w); }
      __builtin_amdgcn_sched_barrier(0);
      q[s] = ld(src(r + 1, s), s);
      __builtin_amdgcn_sched_barrier(0);
    }
    q[NSP] = ld(src(r + 1, NSP), NSP);
    j = jj(r + 1);
  }
  out[blockIdx.x * 1024 + threadIdx.x] = h0 ^ h1 ^ h2 ^ h3;
  if (threadIdx.x == 0) {
    const uint64_t t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    reinterpret_cast<unsigned long long*>(out + (8 << 20))[2 * blockIdx.x] = t1 - t0;
    reinterpret_cast<unsigned long long*>(out + (8 << 20))[2 * blockIdx.x + 1] = r1 - r0;
  }
}

typedef void (*ProbeFn)(const uint8_t*, uint64_t, uint32_t*);
static void run_fn(ProbeFn fn, const char* name, const uint8_t* d, uint64_t npk, uint32_t* out, int blocks);
template <int PAT, int WORK, int NT, int R = 5>
static void run(const char* name, const uint8_t* d, uint64_t npk, uint32_t* out, int blocks) {
  run_fn(probe<PAT, WORK, NT, R>, name, d, npk, out, blocks);
}
static void run_fn(ProbeFn fn, const char* name, const uint8_t* d, uint64_t npk, uint32_t* out, int blocks) {
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  for (int w = 0; w < 3; ++w) hipLaunchKernelGGL(fn, dim3(blocks), dim3(1024), 0, 0, d, npk, out);
  CHECK(hipDeviceSynchronize());
  const int iters = 20;
  CHECK(hipEventRecord(e0, 0));
  for (int w = 0; w < iters; ++w) hipLaunchKernelGGL(fn, dim3(blocks), dim3(1024), 0, 0, d, npk, out);
  CHECK(hipEventRecord(e1, 0));
  CHECK(hipEventSynchronize(e1));
  float ms = 0;
  CHECK(hipEventElapsedTime(&ms, e0, e1));
  const double us = ms * 1000.0 / iters;
  static unsigned long long st[2 * 1024];
  CHECK(hipMemcpy(st, out + (8 << 20), sizeof(unsigned long long) * 2 * blocks, hipMemcpyDeviceToHost));
  double ghz = 0;
  for (int b = 0; b < blocks; ++b) ghz += st[2 * b + 1] ? (double)st[2 * b] / st[2 * b + 1] * 0.1 : 0;
  printf("%-44s %8.1f us  %7.1f GB/s  clk %.2f GHz\n", name, us, npk * 1200.0 / (us * 1e3), ghz / blocks);
}

int main() {
  int cus = 0;
  CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  const uint64_t npk = 1 << 20, bytes = npk * 1200 + 4096;
  uint8_t* d;
  uint32_t* out;
  CHECK(hipMalloc(&d, bytes));
  CHECK(hipMalloc(&out, 64 << 20));
  CHECK(hipMemset(d, 0x5a, bytes));
  if (getenv("PROBE_RANDOM")) {  // random bytes: HBM/fabric power depends on the data
    uint8_t* h = (uint8_t*)malloc(bytes);
    uint64_t x = 88172645463325252ull;
    for (uint64_t i = 0; i + 8 <= bytes; i += 8) { x ^= x << 13; x ^= x >> 7; x ^= x << 17; memcpy(h + i, &x, 8); }
    CHECK(hipMemcpy(d, h, bytes, hipMemcpyHostToDevice));
    free(h);
  }
  printf("CUs=%d, 1M x 1200 B, %s data\n", cus, getenv("PROBE_RANDOM") ? "random" : "0x5a");
  if (getenv("PROBE_SPLIT")) {  // 1M x 1200 B: current shape vs line-split loads, alternating
    for (int rep = 0; rep < 3; ++rep) {
      run_fn(probe_regs<0>, "current shape (register ring)", d, npk, out, cus);
      run_fn(probe_linesplit<2>, "line-split, nt except shared lines", d, npk, out, cus);
      run_fn(probe_linesplit<0>, "line-split, plain", d, npk, out, cus);
      run_fn(probe_linesplit<1>, "line-split, all nt", d, npk, out, cus);
    }
    return 0;
  }
  if (getenv("PROBE_SHARED")) {  // G1 bytes: each line once (P9) vs the kernel's shape, vs P6
    const uint64_t n6 = npk * 1200 / 1280;
    for (int rep = 0; rep < 2; ++rep) {
      run<1, 2, 0, 5>("P1 kernel shape, kernel lookups (DMA)", d, npk, out, cus);
      run_fn(probe_linesplit<0>, "line-split register ring, plain", d, npk, out, cus);
      run<9, 2, 0, 5>("P9 G1 lines once, kernel lookups", d, npk, out, cus);
      run<9, 2, 1, 5>("P9 G1 lines once, kernel lookups nt", d, npk, out, cus);
      run<6, 2, 1, 5>("P6 1280-B lines, kernel lookups nt", d, n6, out, cus);
    }
    return 0;
  }
  if (getenv("PROBE_G1LINES")) {  // 1M x 1200 B, line grid, 11 slots
    run_fn(probe_regs<0>, "P1 kernel lookups, register ring (current shape)", d, npk, out, cus);
    run_fn(probe_regs<1>, "P1 kernel lookups, register ring nt", d, npk, out, cus);
    run_fn(probe_lines<11, 0>, "line grid 11 slots, plain", d, npk, out, cus);
    run_fn(probe_lines<11, 1>, "line grid 11 slots, nt", d, npk, out, cus);
    run_fn(probe_lines<11, 2>, "line grid 11 slots, nt middle", d, npk, out, cus);
    run_fn(probe_lines<11, 1>, "line grid 11 slots, nt (again)", d, npk, out, cus);
    run_fn(probe_regs<0>, "P1 kernel lookups, register ring (again)", d, npk, out, cus);
    return 0;
  }
  if (getenv("PROBE_LINES")) {  // 983,040 x 1280 B = same bytes as 1M x 1200 (GB/s column is exact)
    const uint64_t n6 = npk * 1200 / 1280;
    run<6, 0, 0, 5>("P6 aligned lines xor", d, n6, out, cus);
    run<6, 0, 1, 5>("P6 aligned lines xor nt", d, n6, out, cus);
    run<8, 0, 0, 5>("P8 contiguous xor", d, n6, out, cus);
    run<8, 0, 1, 5>("P8 contiguous xor nt", d, n6, out, cus);
    run<6, 2, 0, 5>("P6 aligned lines kernel lookups", d, n6, out, cus);
    run<6, 2, 1, 5>("P6 aligned lines kernel lookups nt", d, n6, out, cus);
    run<8, 2, 0, 5>("P8 contiguous kernel lookups", d, n6, out, cus);
    run<8, 2, 1, 5>("P8 contiguous kernel lookups nt", d, n6, out, cus);
    run<8, 2, 1, 4>("P8 contiguous kernel lookups nt R=4", d, n6, out, cus);
    return 0;
  }
  if (getenv("PROBE_REGS")) {
    run<1, 0, 0, 5>("P1 xor R=5", d, npk, out, cus);
    run<1, 2, 0, 5>("P1 kernel lookups, LDS-DMA R=5", d, npk, out, cus);
    run_fn(probe_regs<0>, "P1 kernel lookups, register ring", d, npk, out, cus);
    run_fn(probe_regs<1>, "P1 kernel lookups, register ring nt", d, npk, out, cus);
    return 0;
  }
  if (getenv("PROBE_RING")) {
    run<1, 0, 0, 2>("P1 xor R=2", d, npk, out, cus);
    run<1, 0, 0, 3>("P1 xor R=3", d, npk, out, cus);
    run<1, 0, 0, 4>("P1 xor R=4", d, npk, out, cus);
    run<1, 0, 0, 5>("P1 xor R=5", d, npk, out, cus);
    run<1, 0, 0, 6>("P1 xor R=6", d, npk, out, cus);
    run<1, 0, 0, 7>("P1 xor R=7", d, npk, out, cus);
    run<1, 0, 0, 8>("P1 xor R=8", d, npk, out, cus);
    run<2, 0, 1, 5>("P2 aligned xor nt R=5", d, npk, out, cus);
    run<2, 0, 1, 8>("P2 aligned xor nt R=8", d, npk, out, cus);
    run<3, 0, 1, 8>("P3 contiguous xor nt R=8", d, npk, out, cus);
    run<1, 1, 0, 4>("P1 lookups R=4", d, npk, out, cus);
    run<1, 1, 0, 6>("P1 lookups R=6", d, npk, out, cus);
    run<1, 1, 0, 8>("P1 lookups R=8", d, npk, out, cus);
    run<4, 0, 0, 4>("P4 reversed lanes xor R=4", d, npk, out, cus);
    run<4, 0, 0, 5>("P4 reversed lanes xor R=5", d, npk, out, cus);
    run<4, 1, 0, 4>("P4 reversed lanes lookups R=4", d, npk, out, cus);
    run<5, 0, 0, 4>("P5 16 lanes/packet xor R=4", d, npk, out, cus);
    run<5, 0, 0, 6>("P5 16 lanes/packet xor R=6", d, npk, out, cus);
    run<5, 0, 1, 4>("P5 16 lanes/packet xor nt R=4", d, npk, out, cus);
    run<5, 0, 1, 6>("P5 16 lanes/packet xor nt R=6", d, npk, out, cus);
    run<1, 0, 1, 6>("P1 xor nt R=6", d, npk, out, cus);
    run<1, 2, 0, 4>("P1 kernel lookups R=4", d, npk, out, cus);
    run<1, 2, 0, 5>("P1 kernel lookups R=5", d, npk, out, cus);
    return 0;
  }
  run<0, 0, 0>("P0 global stream, xor", d, npk, out, cus);
  run<1, 0, 0>("P1 crc shape (-80), xor", d, npk, out, cus);
  run<2, 0, 0>("P2 crc shape aligned, xor", d, npk, out, cus);
  run<3, 0, 0>("P3 block-contiguous, xor", d, npk, out, cus);
  run<0, 1, 0>("P0 global stream, lookups", d, npk, out, cus);
  run<1, 1, 0>("P1 crc shape (-80), lookups", d, npk, out, cus);
  run<2, 1, 0>("P2 crc shape aligned, lookups", d, npk, out, cus);
  run<3, 1, 0>("P3 block-contiguous, lookups", d, npk, out, cus);
  run<1, 0, 1>("P1 crc shape (-80), xor, nt", d, npk, out, cus);
  run<3, 0, 1>("P3 block-contiguous, xor, nt", d, npk, out, cus);
  run<1, 1, 1>("P1 crc shape (-80), lookups, nt", d, npk, out, cus);
  return 0;
}
