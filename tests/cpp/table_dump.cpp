// Host build of the kernels' table generator (rusty_enet_amd/csrc/crc32_ops.hpp):
// prints the Sarwate table the kernels use and op[0][3] (M32 applied to b << 24,
// which the LDS block stores as the byte-step table, crc32_layout.hpp), one hex
// entry per line each.  tests/test_table_pin.py hashes them against the pin of
// src/crc32.rs:1-34.
#include <stdio.h>

#include "../../rusty_enet_amd/csrc/crc32_ops.hpp"

int main() {
  for (int i = 0; i < 256; ++i) printf("%08x\n", enet_crc::kOpTables.sarwate[i]);
  for (int i = 0; i < 256; ++i) printf("%08x\n", enet_crc::kOpTables.op[0][3][i]);
  return 0;
}
