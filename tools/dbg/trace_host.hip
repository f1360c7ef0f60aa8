// Host run of the debug decoder trace for one input (compare with tools/dbg/range_dbg.py on the GPU).
#define RC_DEBUG_EXITS 1
#include <stdio.h>
#include <string.h>
#include <vector>
#include "../../rusty_enet_amd/csrc/range_coder.hip"
extern "C" {
typedef struct oracle_iov { const uint8_t* data; size_t len; } oracle_iov;
size_t oracle_range_compress(const oracle_iov* bufs, size_t nbufs, size_t in_limit, uint8_t* out, size_t out_limit);
}
int main(int argc, char** argv) {
  const char* x = argc > 1 ? argv[1] : "hello hello hello world";
  std::vector<uint8_t> c(4096), o(8192, 0);
  oracle_iov one = {(const uint8_t*)x, strlen(x)};
  size_t n = oracle_range_compress(&one, 1, strlen(x), c.data(), c.size());
  std::vector<enet_crc::Sym> arena(4096);
  enet_crc::Model m; m.a = arena.data();
  uint32_t r = enet_crc::decompress_one(m, c.data(), (uint32_t)n, o.data(), 8192);
  printf("ret=%x\n", r);
  for (int k = 0; k < 16; ++k) {
    const enet_crc::Sym* y = (const enet_crc::Sym*)(o.data() + 4096 + 16 * k);
    printf("sym%2d v=%3u c=%3u u=%5u L=%u R=%u S=%u E=%u T=%u P=%u\n", k, y->value, y->count, y->under, y->left, y->right, y->symbols, y->escapes, y->total, y->parent);
  }
  for (int k = 0; k < 8; ++k) {
    uint32_t* t = (uint32_t*)(o.data() + 2048 + 16 * k);
    printf("%d v=%c ctx=%u pred=%u low=%08x range=%08x code=%08x\n", k, t[0] & 0xFF, (t[0] >> 8) & 0xFFF, t[0] >> 20, t[1], t[2], t[3]);
  }
}
// (appended) arena dump printer lives in main via env
