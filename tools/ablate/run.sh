#!/usr/bin/env bash
# Build ablation variants of the kernel source (here, CPU) -> tools/ablate/bin/*.
# Each variant = a sed patch of crc32_kernels.hip.  Run them on the GPU with
#   gpurun -- 'for b in tools/ablate/bin/*; do timeout -k 5 60 $b; done'
set -eu
cd "$(dirname "$0")"
mkdir -p bin gen
SRC=../../rusty_enet_amd/csrc/crc32_kernels.hip
build() {  # name, python-replacement-script
  local name=$1; shift
  python3 - "$SRC" "gen/$name.hip" "$name" "$@" <<'PY'
import sys
src, dst, name = sys.argv[1:4]
s = open(src).read()
for pair in sys.argv[4:]:
    a, b = pair.split('=>', 1)
    assert a in s, (name, a)
    s = s.replace(a, b)
s = s.replace('#include "crc32_geometry.hpp"', '#include "../../../rusty_enet_amd/csrc/crc32_geometry.hpp"')
s = s.replace('#include "crc32_kernels.hpp"', '#include "../../../rusty_enet_amd/csrc/crc32_kernels.hpp"')
s = s.replace('#include "crc32_ops.hpp"', '#include "../../../rusty_enet_amd/csrc/crc32_ops.hpp"')
open(dst, 'w').write('#define VARIANT_NAME "%s"\n' % name + s)
PY
  cp "gen/$name.hip" gen/variant.hip
  (cd gen && /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++20 -I. -o "../bin/$name" ../ablate_main.hip)
}
build base
build no_mem 'q[s] = load_chunk(pn + (uint64_t)kBytesPerStep * s);=>q[s] = load_chunk(c.dummy + 16u * c.k);' \
  'q[s] = load_chunk(pa + (uint64_t)kBytesPerStep * s);=>q[s] = load_chunk(c.dummy + 16u * c.k);'
build no_lookup 'return xor3(xor3(lds_at(lds, a0), lds_at(lds, a1 + 128u), lds_at(lds, a2)), lds_at(lds, a3 + 128u), w);=>return xor3(xor3(a0, a1, a2), a3, w);'
build no_lookup_no_mem 'return xor3(xor3(lds_at(lds, a0), lds_at(lds, a1 + 128u), lds_at(lds, a2)), lds_at(lds, a3 + 128u), w);=>return xor3(xor3(a0, a1, a2), a3, w);' \
  'q[s] = load_chunk(pn + (uint64_t)kBytesPerStep * s);=>q[s] = load_chunk(c.dummy + 16u * c.k);' \
  'q[s] = load_chunk(pa + (uint64_t)kBytesPerStep * s);=>q[s] = load_chunk(c.dummy + 16u * c.k);'
build lds_only 'return xor3(xor3(lds_at(lds, a0), lds_at(lds, a1 + 128u), lds_at(lds, a2)), lds_at(lds, a3 + 128u), w);=>return xor3(xor3(lds_at(lds, lp0), lds_at(lds, lp0 + 128u), lds_at(lds, lp1)), lds_at(lds, lp1 + 128u), w ^ a0 ^ a1 ^ a2 ^ a3);'
ls -la bin
