#!/usr/bin/env bash
# Build ablation variants of the kernel source (here, CPU) -> tools/ablate/bin/*.
# Each variant = a text patch of crc32_kernels.hip.  Run them on the GPU with
#   gpurun -- bash scripts/gpu_ablate.sh
# (ENET_CRC_UNIFORM=regs selects the register-ring uniform kernel in every variant.)
set -eu
cd "$(dirname "$0")"
mkdir -p bin gen
SRC=../../rusty_enet_amd/csrc/crc32_kernels.hip
build() {  # name, 'old=>new' replacements...
  local name=$1; shift
  python3 - "$SRC" "gen/$name.hip" "$name" "$@" <<'PY'
import sys
src, dst, name = sys.argv[1:4]
s = open(src).read()
for pair in sys.argv[4:]:
    a, b = pair.split('=>', 1)
    once = a.startswith('1:')
    a = a[2:] if once else a
    assert a in s, (name, a)
    s = s.replace(a, b, 1) if once else s.replace(a, b)
for h in ("crc32_geometry.hpp", "crc32_kernels.hpp", "crc32_ops.hpp", "crc32_layout.hpp"):
    s = s.replace('#include "%s"' % h, '#include "../../../rusty_enet_amd/csrc/%s"' % h)
open(dst, 'w').write('#define VARIANT_NAME "%s"\n' % name + s)
PY
  cp "gen/$name.hip" gen/variant.hip
  (cd gen && /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++20 -I. -w -o "../bin/$name" ../ablate_main.hip)
}
NO_LOOKUP='return xor3(xor3(lds_at(lds, a0), lds_at(lds, a1), lds_at(lds, a2)), lds_at(lds, a3), w);=>return xor3(xor3(a0, a1, a2), a3, w);'
DMA_NOMEM='__builtin_amdgcn_global_load_lds((const void*)src,=>__builtin_amdgcn_global_load_lds((const void*)(c.dummy + 16u * c.k + 0 * src),'
REGS_NOMEM1='q[s] = load_chunk(pn + (uint64_t)kBytesPerStep * s);=>q[s] = load_chunk(c.dummy + 16u * c.k);'
REGS_NOMEM2='q[s] = load_chunk(pa + (uint64_t)kBytesPerStep * s);=>q[s] = load_chunk(c.dummy + 16u * c.k);'
DMA_NT='(LdsVoid*)&ring[q][wv][0], 16, 0, 0);=>(LdsVoid*)&ring[q][wv][0], 16, 0, 2);'
DMA_SC='(LdsVoid*)&ring[q][wv][0], 16, 0, 0);=>(LdsVoid*)&ring[q][wv][0], 16, 0, 3);'
COMB_DMA='uint32_t reg = combine_streams(lds, h0, h1, h2, h3);
    if (z != 0 && c.k == 0)=>uint32_t reg = h0 ^ h1 ^ h2 ^ h3;
    if (z != 0 && c.k == 0)'
NOLK_DMA='"ds_read_b32 %5, %5\n\tds_read_b32 %6, %6\n\tds_read_b32 %7, %7\n\tds_read_b32 %8, %8\n\t"
      "ds_read_b32 %9, %9\n\tds_read_b32 %10, %10\n\tds_read_b32 %11, %11\n\tds_read_b32 %12, %12\n\t"
      "ds_read_b32 %13, %13\n\tds_read_b32 %14, %14\n\tds_read_b32 %15, %15\n\tds_read_b32 %16, %16\n\t"
      "ds_read_b32 %17, %17\n\tds_read_b32 %18, %18\n\tds_read_b32 %19, %19\n\tds_read_b32 %20, %20\n\t"=>'
HALFLK_DMA='"ds_read_b32 %13, %13\n\tds_read_b32 %14, %14\n\tds_read_b32 %15, %15\n\tds_read_b32 %16, %16\n\t"
      "ds_read_b32 %17, %17\n\tds_read_b32 %18, %18\n\tds_read_b32 %19, %19\n\tds_read_b32 %20, %20\n\t"=>'
NOPERM='for (int t = 0; t < 4; ++t) a[4 * j + t] = __builtin_amdgcn_perm(hs[j], lk.lp, lk.sel[t]);=>for (int t = 0; t < 4; ++t) a[4 * j + t] = hs[j];'
STATIC1='1:uint32_t q = 0;  // ring position of the slot being consumed (wave-uniform)=>uint32_t q = 0; uint32_t nfetch = 0;'
STATIC2='1:if (lane == 0) d = lds_fetch_add_one(&next_dispatch);=>d = kWavesPerBlock * (kLook + nfetch++) + wv;'
NODUMMY='return none0 || is_below(pb) ? c.dummy : pb + (uint64_t)rel0;=>return (int64_t)(pb - u.base) + rel0 < 0 ? c.dummy : pb + (uint64_t)rel0;'
NOFILL='if (threadIdx.x == 0) next_dispatch = kWavesPerBlock * kLook;
  fill_lds(lds);=>if (threadIdx.x == 0) next_dispatch = kWavesPerBlock * kLook;'
SMALL='constexpr uint32_t kLdsDwords = kInvTopDword + 64;=>constexpr uint32_t kLdsDwords = 1024;'
RING6='constexpr int kDmaRing = 4; =>constexpr int kDmaRing = 6; '
RING8='constexpr int kDmaRing = 4; =>constexpr int kDmaRing = 8; '
R5A='constexpr int kSmallSets = 1 + kTreeLevels;=>constexpr int kSmallSets = kTreeLevels;'
R5B='if (k == 4u) t = apply_small(lds + kMainDwords + 3072, y);=>if (k == 4u) t = apply_small(lds + kMainDwords + 2048, apply_small(lds + kMainDwords + 2048, y));'
R5C='constexpr int kDmaRing = 4; =>constexpr int kDmaRing = 5; '
R5D='1:__global__ __launch_bounds__(kBlock) void crc32_ragged_dma_kernel(RaggedDmaBatch b, uint32_t* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) uint32_t lds[kLdsDwords];
  __shared__ __attribute__((aligned(16))) u32x4 ring[kDmaRing][kWavesPerBlock][64];=>__global__ __launch_bounds__(kBlock) void crc32_ragged_dma_kernel(RaggedDmaBatch b, uint32_t* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) uint32_t lds[kLdsDwords];
  __shared__ __attribute__((aligned(16))) u32x4 ring[4][kWavesPerBlock][64];'
if [ "${ABLATE_SET:-}" = basic ]; then
  build base
  ls -la bin; exit 0
fi
if [ "${ABLATE_SET:-}" = r5 ]; then
  build base
  build tree2 "$R5A" "$R5B"
  build ring5 "$R5A" "$R5B" "$R5C" "$R5D"
  ls -la bin; exit 0
fi
if [ "${ABLATE_SET:-}" = ring ]; then
  build skel_nofill "$NOLK_DMA" "$COMB_DMA" "$NOPERM" "$NOFILL"
  build skel_small_r4 "$NOLK_DMA" "$COMB_DMA" "$NOPERM" "$NOFILL" "$SMALL"
  build skel_small_r6 "$NOLK_DMA" "$COMB_DMA" "$NOPERM" "$NOFILL" "$SMALL" "$RING6"
  build skel_small_r8 "$NOLK_DMA" "$COMB_DMA" "$NOPERM" "$NOFILL" "$SMALL" "$RING8"
  ls -la bin; exit 0
fi
if [ "${ABLATE_SET:-}" = fill ]; then
  build base
  build skel_noperm "$NOLK_DMA" "$COMB_DMA" "$NOPERM"
  build skel_nofill "$NOLK_DMA" "$COMB_DMA" "$NOPERM" "$NOFILL"
  build base_nofill "$NOFILL"
  ls -la bin; exit 0
fi
if [ "${ABLATE_SET:-}" = bisect ]; then
  build base
  build skel_noperm "$NOLK_DMA" "$COMB_DMA" "$NOPERM"
  build skel_static "$NOLK_DMA" "$COMB_DMA" "$NOPERM" "$STATIC1" "$STATIC2"
  build skel_nodummy "$NOLK_DMA" "$COMB_DMA" "$NOPERM" "$NODUMMY"
  build skel_static_nodummy "$NOLK_DMA" "$COMB_DMA" "$NOPERM" "$STATIC1" "$STATIC2" "$NODUMMY"
  build base_static "$STATIC1" "$STATIC2"
  build base_nodummy "$NODUMMY"
  ls -la bin; exit 0
fi
if [ "${ABLATE_SET:-}" = skel ]; then
  build base
  build no_lookup_comb_trivial "$NOLK_DMA" "$COMB_DMA"
  build skel_noperm "$NOLK_DMA" "$COMB_DMA" "$NOPERM"
  build no_mem "$DMA_NOMEM"
  ls -la bin; exit 0
fi
if [ "${ABLATE_SET:-}" = lk ]; then
  build base
  build no_lookup_dma "$NOLK_DMA"
  build half_lookup_dma "$HALFLK_DMA"
  build comb_trivial_dma "$COMB_DMA"
  build no_lookup_comb_trivial "$NOLK_DMA" "$COMB_DMA"
  ls -la bin; exit 0
fi
if [ "${ABLATE_SET:-}" = comb ]; then
  build base
  build comb_trivial_dma "$COMB_DMA"
  build no_mem "$DMA_NOMEM" "$REGS_NOMEM1" "$REGS_NOMEM2"
  build no_mem_comb_trivial "$DMA_NOMEM" "$REGS_NOMEM1" "$REGS_NOMEM2" "$COMB_DMA"
  ls -la bin; exit 0
fi
if [ "${ABLATE_SET:-}" = nt ]; then
  build base
  build nt "$DMA_NT"
  build nt_sc0 "$DMA_SC"
  build no_lookup "$NO_LOOKUP"
  build no_lookup_nt "$NO_LOOKUP" "$DMA_NT"
  ls -la bin; exit 0
fi
build base
build no_lookup "$NO_LOOKUP"
build no_mem "$DMA_NOMEM" "$REGS_NOMEM1" "$REGS_NOMEM2"
build no_lookup_no_mem "$NO_LOOKUP" "$DMA_NOMEM" "$REGS_NOMEM1" "$REGS_NOMEM2"
build comb_trivial 'uint32_t reg = combine_streams(lds, h0, h1, h2, h3);=>uint32_t reg = h0 ^ h1 ^ h2 ^ h3;'
STAMP1='__device__ const OpTables g_op_tables = kOpTables;=>__device__ const OpTables g_op_tables = kOpTables;
#define STAMPS 1
__device__ unsigned long long g_stamp[6 * 8192];'
STAMP2='const u32x4 v = read_landed_slot<kDmaRing - 1>(ring0 + q * kRingStride + lane * 16u);=>const uint64_t st0 = __builtin_readcyclecounter(); uint64_t st1; u32x4 v;
      asm volatile("s_waitcnt vmcnt(%2)\n\ts_memtime %1\n\tds_read_b128 %0, %3\n\ts_waitcnt lgkmcnt(0)" : "=v"(v), "=&s"(st1) : "i"(kDmaRing - 1), "v"(ring0 + q * kRingStride + lane * 16u) : "memory");
      t_vm += st1 - st0; t_ds += __builtin_readcyclecounter() - st1;'
STAMP3='uint32_t res = 0, j = 0;=>uint32_t res = 0, j = 0; uint64_t t_vm = 0, t_ds = 0, t_comb = 0; const uint64_t t_start = __builtin_readcyclecounter(); const uint64_t rt_start = __builtin_amdgcn_s_memrealtime();'
STAMP4='    uint32_t reg = combine_streams(lds, h0, h1, h2, h3);
    if constexpr (kTail) reg = tail_steps(lds, reg, tw, ntail, 0);
    const uint32_t crc=>    const uint64_t sc0 = __builtin_readcyclecounter();
    uint32_t reg = combine_streams(lds, h0, h1, h2, h3);
    if constexpr (kTail) reg = tail_steps(lds, reg, tw, ntail, 0);
    const uint32_t crc'
STAMP5='    // Lane 8g+j keeps the checksum=>    t_comb += __builtin_readcyclecounter() - sc0;
    // Lane 8g+j keeps the checksum'
STAMP6='  __builtin_amdgcn_s_waitcnt(0);
}=>  { const uint32_t wave = blockIdx.x * 16 + wv; if (lane == 0) { g_stamp[wave * 4] = t_vm; g_stamp[wave * 4 + 1] = t_ds; g_stamp[wave * 4 + 2] = t_comb; g_stamp[wave * 4 + 3] = __builtin_readcyclecounter() - t_start; g_stamp[32768 + wave] = __builtin_amdgcn_s_memrealtime() - rt_start; g_stamp[40960 + wave] = rt_start; } }
  __builtin_amdgcn_s_waitcnt(0);
}'
build stamps "$STAMP1" "$STAMP2" "$STAMP3" "$STAMP4" "$STAMP5" "$STAMP6"
build stamps_no_mem "$STAMP1" "$STAMP2" "$STAMP3" "$STAMP4" "$STAMP5" "$STAMP6" "$DMA_NOMEM"
ls -la bin
