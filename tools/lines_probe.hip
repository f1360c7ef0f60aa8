// Probe (tooling, round 6): the ragged jobs kernel's load stream with its lookups, on real
// packet layouts, with the 256-B pair pieces anchored either at each packet's end (the
// product: pieces end at the packet's 4-byte-grid end, so a piece straddles 3 lines) or at
// 128-B lines (each compute slot is one whole line of the packet: a packet of L bytes from
// offset o reads lines o >> 7 .. (o + L - 1) >> 7, the boundary lines that two neighbours
// share included), and with or without the non-temporal hint on the DMAs.  tools/dma_shape
// (round 6) measured aligned + non-temporal 8 x 128-B pieces at 316 us for 1392-B packets
// against 383 us end-anchored, but its aligned pieces skip each packet's last partial line
// (so no line is read twice) and it does no lookups; this probe reads exactly the lines the
// arithmetic would need.
//
// Per wave: rounds of 8 consecutive packets of the batch (static: round gw + j * nw), NS =
// max over the 8 of their slot counts rounded up to even, slot s of packet g = 128 B ending
// NS - 1 - s lines before its last one (line anchor) or 128 (NS - s) B before its end (end
// anchor); slots before a packet read the 64-B zero chunk.  Pair P = slots 2P, 2P + 1 as two
// LDS-DMA instructions of 4 packets x 256 B into a 2-pair-slot ring (as the product); the
// next round's first 2 pairs are issued by the round before.  Per landed 16 B the lane does one
// pass of the product's lookups (16 ds_read_b32 from the replicated block).  NT policy: 0 none,
// 1 every DMA, 2 every DMA but those of a round's first two pairs and its last pair (the
// pairs that hold lines shared with a neighbour).  Host-side round geometry: per round NS and
// per packet (first line, last line, end) as u64 in HBM, read one round ahead.
//   hipcc --offload-arch=gfx950 -O3 -std=c++20 -o tools/lines_probe tools/lines_probe.hip
//   tools/lines_probe <layout: L | frag | g2> [n]
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <random>
#include <vector>

typedef __attribute__((address_space(3))) void LdsVoid;
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

constexpr int kWaves = 16;
constexpr int kLdsBytes = 159 * 1024;
constexpr int kTableBytes = 64 * 1024;
__device__ __attribute__((aligned(64))) const uint32_t g_zero[64] = {0};

struct PacketGeo {
  uint64_t first_line;  // byte address of the packet's first line
  uint64_t last_line;   // byte address of its last line
  uint64_t end;         // its 4-byte-grid end
  uint64_t start;
};

template <int N>
__device__ __forceinline__ u32x4 read_landed(uint32_t addr) {
  u32x4 v;
  asm volatile("s_waitcnt vmcnt(%1)\n\tds_read_b128 %0, %2\n\ts_waitcnt lgkmcnt(0)"
               : "=v"(v)
               : "i"(N), "v"(addr)
               : "memory");
  return v;
}

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

// kLine: pieces anchored at lines (else at the packet end); kNT: 0 none, 1 all, 2 interior pairs.
template <bool kLine, int kNT>
__global__ __launch_bounds__(1024) void lines_kernel(const PacketGeo* __restrict__ geo, const uint32_t* __restrict__ rns,
                                                     uint64_t rounds, uint32_t* out) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[kLdsBytes];
  const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  for (uint32_t x = threadIdx.x; x < kTableBytes / 4; x += 1024) reinterpret_cast<uint32_t*>(lds)[x] = x * 2654435761u;
  __syncthreads();
  if ((uint32_t)(uintptr_t)(LdsVoid*)lds != 0) __builtin_trap();
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
  const uint64_t gw = (uint64_t)blockIdx.x * kWaves + wv, nw = (uint64_t)gridDim.x * kWaves;
  const uint64_t my_rounds = gw < rounds ? (rounds - gw + nw - 1) / nw : 0;
  if (my_rounds == 0) return;
  const uint32_t ring0 = kTableBytes + wv * 2048u;  // pair slot q at ring0 + q * 32 KiB
  auto slot_addr = [&](uint32_t q) { return ring0 + q * (kWaves * 2048u); };
  // This lane's two DMA packets (4 i + lane / 16) of round j, and its 16-B offset in a 256-B piece.
  const uint32_t off16 = 16u * (lane & 15u);
  struct Plan {
    uint64_t a0, a1, lo0, lo1;  // piece-0 address of each DMA packet; the lowest real address
    uint32_t ns;
  };
  auto plan_of = [&](uint64_t j) -> Plan {
    Plan p;
    const uint64_t r = gw + j * nw;
    if (j >= my_rounds) {
      p.ns = 4;  // past this wave's rounds: every chunk is the zero chunk
      p.a0 = p.a1 = 0;
      p.lo0 = p.lo1 = ~0ull;
      return p;
    }
    p.ns = rns[r];
    const PacketGeo g0 = geo[8 * r + (lane >> 4)], g1 = geo[8 * r + 4 + (lane >> 4)];
    if (kLine) {
      p.a0 = g0.last_line - 128u * (p.ns - 1) + off16;
      p.a1 = g1.last_line - 128u * (p.ns - 1) + off16;
      p.lo0 = g0.first_line;
      p.lo1 = g1.first_line;
    } else {
      p.a0 = g0.end - 128u * p.ns + off16;
      p.a1 = g1.end - 128u * p.ns + off16;
      p.lo0 = (g0.start & ~3ull) - 15;  // a chunk is real once its 16 B reach the first word
      p.lo1 = (g1.start & ~3ull) - 15;
    }
    return p;
  };
  auto issue = [&](const Plan& p, uint32_t P, uint32_t q) {
    const uint64_t s0 = p.a0 + 256u * P, s1 = p.a1 + 256u * P;
    const void* x0 = s0 >= p.lo0 ? (const void*)s0 : (const void*)g_zero;
    const void* x1 = s1 >= p.lo1 ? (const void*)s1 : (const void*)g_zero;
    LdsVoid* d = (LdsVoid*)(lds + slot_addr(q));
    const bool nt = kNT == 1 || (kNT == 2 && P >= 2 && P + 1 < p.ns / 2);
    if (nt) {
      __builtin_amdgcn_global_load_lds(x0, d, 16, 0, 2);
      __builtin_amdgcn_global_load_lds(x1, (LdsVoid*)((char*)d + 1024), 16, 0, 2);
    } else {
      __builtin_amdgcn_global_load_lds(x0, d, 16, 0, 0);
      __builtin_amdgcn_global_load_lds(x1, (LdsVoid*)((char*)d + 1024), 16, 0, 0);
    }
  };
  Plan cur = plan_of(0), nxt = plan_of(1);
  issue(cur, 0, 0);
  issue(cur, 1, 1);
  u32x4 h = {lane, 0, 0, 0};
  uint32_t q = 0;
  for (uint64_t j = 0; j < my_rounds; ++j) {
    const uint32_t np = cur.ns / 2;
    for (uint32_t P = 0; P < np; ++P) {
      const u32x4 v0 = read_landed<2>(slot_addr(q) + 16 * lane);
      u32x4 v1;
      asm volatile("ds_read_b128 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(v1) : "v"(slot_addr(q) + 1024 + 16 * lane) : "memory");
      const uint32_t f = P + 2;
      if (f < np)
        issue(cur, f, q);
      else
        issue(nxt, f - np, q);
      q ^= 1u;
      lookup_pass(lk, h, v0);
      lookup_pass(lk, h, v1);
    }
    cur = nxt;
    nxt = plan_of(j + 2);
  }
  __builtin_amdgcn_s_waitcnt(0);
  out[(blockIdx.x * 1024 + threadIdx.x)] = h.x ^ h.y ^ h.z ^ h.w;
}

#define CHECK(x)                                                             \
  do {                                                                       \
    hipError_t e_ = (x);                                                     \
    if (e_ != hipSuccess) {                                                  \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                \
      return 2;                                                              \
    }                                                                        \
  } while (0)

struct Variant {
  const char* name;
  bool line;
  void (*launch)(int, const PacketGeo*, const uint32_t*, uint64_t, uint32_t*);
};
template <bool kLine, int kNT>
void launch_v(int grid, const PacketGeo* g, const uint32_t* r, uint64_t rounds, uint32_t* out) {
  hipLaunchKernelGGL((lines_kernel<kLine, kNT>), dim3(grid), dim3(1024), 0, 0, g, r, rounds, out);
}

int main(int argc, char** argv) {
  const char* layout = argc > 1 ? argv[1] : "1392";
  std::vector<uint32_t> len;
  uint64_t n = argc > 2 ? strtoull(argv[2], nullptr, 10) : 0;
  if (!strcmp(layout, "frag")) {
    if (!n) n = 32768;
    for (uint64_t i = 0; i < n; ++i) {
      for (int k = 0; k < 48; ++k) len.push_back(1392);
      len.push_back(288);
    }
  } else if (!strcmp(layout, "g2")) {
    if (!n) n = 1 << 20;
    std::mt19937_64 rng(1234);
    for (uint64_t i = 0; i < n; ++i) len.push_back(64 + (uint32_t)(rng() % 1329));
  } else {
    const uint32_t L = (uint32_t)atoi(layout);
    if (!n) n = 1 << 20;
    len.assign(n, L);
  }
  while (len.size() % 8) len.push_back(0);
  const uint64_t np = len.size(), rounds = np / 8;
  uint64_t total = 0;
  for (uint32_t l : len) total += l;
  uint8_t* buf = nullptr;
  CHECK(hipMalloc(&buf, total + 16384));
  CHECK(hipMemset(buf, 0x5a, total + 16384));
  const uint64_t base = (uint64_t)(uintptr_t)buf + 4096;  // line-aligned
  // Rounds as the job sort makes them: packets of one job sorted by step count (jobs of 256).
  std::vector<uint64_t> off(np);
  {
    uint64_t o = 0;
    for (uint64_t i = 0; i < np; ++i) {
      off[i] = o;
      o += len[i];
    }
  }
  std::vector<uint64_t> order(np);
  for (uint64_t i = 0; i < np; ++i) order[i] = i;
  for (uint64_t j0 = 0; j0 < np; j0 += 256) {
    const uint64_t j1 = std::min<uint64_t>(np, j0 + 256);
    std::stable_sort(order.begin() + j0, order.begin() + j1, [&](uint64_t a, uint64_t b) {
      return (len[a] + 127) / 128 < (len[b] + 127) / 128;
    });
  }
  std::vector<PacketGeo> geo(np);
  std::vector<uint32_t> rns(rounds);
  for (uint64_t r = 0; r < rounds; ++r) {
    uint32_t mx_line = 0, mx_end = 0;
    for (int g = 0; g < 8; ++g) {
      const uint64_t p = order[8 * r + g];
      const uint64_t s = base + off[p], e = s + len[p], e4 = (e + 3) & ~3ull;
      PacketGeo pg;
      pg.start = s;
      pg.end = e4;
      pg.first_line = s & ~127ull;
      pg.last_line = len[p] ? (e - 1) & ~127ull : pg.first_line;
      geo[8 * r + g] = pg;
      const uint32_t lines = len[p] ? (uint32_t)((pg.last_line - pg.first_line) / 128 + 1) : 0;
      const uint32_t steps = len[p] ? (uint32_t)((e4 - (s & ~3ull) + 127) / 128) : 0;
      mx_line = std::max(mx_line, lines);
      mx_end = std::max(mx_end, steps);
    }
    rns[r] = std::max<uint32_t>(4, (std::max(mx_line, mx_end) + 1) & ~1u);  // one NS fits both anchors
  }
  PacketGeo* d_geo = nullptr;
  uint32_t *d_rns = nullptr, *out = nullptr;
  CHECK(hipMalloc(&d_geo, geo.size() * sizeof(PacketGeo)));
  CHECK(hipMalloc(&d_rns, rns.size() * 4));
  hipDeviceProp_t prop;
  CHECK(hipGetDeviceProperties(&prop, 0));
  const int grid = prop.multiProcessorCount;
  CHECK(hipMalloc(&out, (size_t)grid * 1024 * 4));
  CHECK(hipMemcpy(d_geo, geo.data(), geo.size() * sizeof(PacketGeo), hipMemcpyHostToDevice));
  CHECK(hipMemcpy(d_rns, rns.data(), rns.size() * 4, hipMemcpyHostToDevice));
  // The anchors need different slot counts; one NS per round fits both (the wider of the two),
  // so the end-anchored rows read at most one extra zero slot per round.
  const Variant vs[] = {
      {"end-anchored, plain (product)", false, launch_v<false, 0>},
      {"end-anchored, nt interior", false, launch_v<false, 2>},
      {"line-anchored, plain", true, launch_v<true, 0>},
      {"line-anchored, nt all", true, launch_v<true, 1>},
      {"line-anchored, nt interior", true, launch_v<true, 2>},
  };
  const int nv = sizeof(vs) / sizeof(vs[0]);
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  printf("layout=%s packets=%llu bytes=%llu rounds=%llu grid=%d\n", layout, (unsigned long long)np,
         (unsigned long long)total, (unsigned long long)rounds, grid);
  fflush(stdout);
  for (int w = 0; w < 60; ++w) vs[w % nv].launch(grid, d_geo, d_rns, rounds, out);
  CHECK(hipGetLastError());
  CHECK(hipDeviceSynchronize());
  std::vector<std::vector<float>> us(nv);
  const int kBlocks = 8, kLaunches = 20;
  for (int blk = 0; blk < kBlocks; ++blk)
    for (int j = 0; j < nv; ++j) {
      const int s = blk % 2 ? nv - 1 - j : j;
      vs[s].launch(grid, d_geo, d_rns, rounds, out);
      CHECK(hipEventRecord(e0, 0));
      for (int it = 0; it < kLaunches; ++it) vs[s].launch(grid, d_geo, d_rns, rounds, out);
      CHECK(hipEventRecord(e1, 0));
      CHECK(hipEventSynchronize(e1));
      float ms = 0;
      CHECK(hipEventElapsedTime(&ms, e0, e1));
      us[s].push_back(1000.f * ms / kLaunches);
    }
  for (int s = 0; s < nv; ++s) {
    std::vector<float> v = us[s];
    std::sort(v.begin(), v.end());
    const float med = 0.5f * (v[kBlocks / 2 - 1] + v[kBlocks / 2]);
    printf("%-32s median %8.1f us  (%7.1f-%7.1f)  %.3f of 8 TB/s\n", vs[s].name, med, v.front(), v.back(),
           total / (med * 1e-6) / 8e12);
  }
  return 0;
}
