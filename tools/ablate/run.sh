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
ls -la bin
