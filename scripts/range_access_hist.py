"""Arena access profile of the range coder (analysis only, CPU).

Builds an instrumented copy of oracle/range_coder_oracle.c in a temp directory (every
symbol access counted by arena index), compresses ragged U{64..1392} packets of the
bench's compressible bytes, and prints the accesses per input byte and the share of
accesses that fall on the first K symbols of the arena (what an LDS cache of the
K first-allocated symbols per coder would catch).  DESIGN.md §11.
"""
import os
import re
import subprocess
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
from _data import enet_like_bytes  # noqa: E402

MAIN = r"""
#include <stdio.h>
#include <stdlib.h>
#include <stdint.h>
typedef struct { const uint8_t* data; size_t len; } oracle_iov;
size_t oracle_range_compress(const oracle_iov*, size_t, size_t, uint8_t*, size_t);
extern unsigned long long HIST[4096];
int main(void) {
  FILE* f = fopen("data.bin", "rb"); fseek(f, 0, 2); long n = ftell(f); fseek(f, 0, 0);
  uint8_t* d = malloc(n); if (fread(d, 1, n, f) != (size_t)n) return 1; fclose(f);
  FILE* g = fopen("lens.bin", "rb"); fseek(g, 0, 2); long m = ftell(g) / 4; fseek(g, 0, 0);
  uint32_t* L = malloc(m * 4); if (fread(L, 4, m, g) != (size_t)m) return 1;
  uint8_t out[8192]; size_t off = 0, tot = 0;
  for (long i = 0; i < m; i++) { oracle_iov v = {d + off, L[i]}; tot += oracle_range_compress(&v, 1, L[i], out, sizeof out); off += L[i]; }
  unsigned long long all = 0; for (int i = 0; i < 4096; i++) all += HIST[i];
  printf("packets %ld bytes %zu accesses/byte %.2f compressed/input %.3f\n", m, off, (double)all / off, (double)tot / off);
  int Ks[] = {1, 2, 4, 8, 16, 32, 64, 128, 256, 512, 1024}; unsigned long long c = 0; int k = 0;
  for (int i = 0; i < 4096; i++) { c += HIST[i]; if (k < 11 && i + 1 == Ks[k]) { printf("first %4d symbols: %.3f of accesses\n", Ks[k], (double)c / all); k++; } }
  return 0;
}
"""


def main(packets: int = 20000) -> None:
    src = open(os.path.join(ROOT, "oracle", "range_coder_oracle.c")).read()
    src = src.replace("#include <string.h>",
                      "#include <string.h>\nunsigned long long HIST[4096];\n"
                      "static inline size_t H(size_t i) { HIST[i]++; return i; }")
    src = re.sub(r"c->s\[([^\]]+)\]", r"c->s[H(\1)]", src)
    src = re.sub(r"c\.s\[([^\]]+)\]", r"c.s[H(\1)]", src)
    with tempfile.TemporaryDirectory() as tmp:
        open(os.path.join(tmp, "oracle_hist.c"), "w").write(src)
        open(os.path.join(tmp, "main.c"), "w").write(MAIN)
        rng = np.random.default_rng(1)
        lens = rng.integers(64, 1393, size=packets).astype(np.uint32)
        enet_like_bytes(7, int(lens.sum())).tofile(os.path.join(tmp, "data.bin"))
        lens.tofile(os.path.join(tmp, "lens.bin"))
        subprocess.run(["gcc", "-O2", "-o", "hist", "main.c", "oracle_hist.c"], cwd=tmp, check=True)
        print(subprocess.run(["./hist"], cwd=tmp, check=True, capture_output=True, text=True).stdout, end="")


if __name__ == "__main__":
    main()
