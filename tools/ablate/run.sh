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
    assert a in s, (name, a)
    s = s.replace(a, b)
for h in ("crc32_geometry.hpp", "crc32_kernels.hpp", "crc32_ops.hpp"):
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
