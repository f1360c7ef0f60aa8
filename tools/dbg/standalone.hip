// Standalone GPU check of the range decoder (no torch): arena zeroed vs garbage.
#include <stdio.h>
#include <string.h>
#include <vector>
#include "../../rusty_enet_amd/csrc/range_coder.hip"
extern "C" {
typedef struct oracle_iov { const uint8_t* data; size_t len; } oracle_iov;
size_t oracle_range_compress(const oracle_iov* bufs, size_t nbufs, size_t in_limit, uint8_t* out, size_t out_limit);
}
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); return 2; } } while (0)
int main() {
  const char* x = "hello hello hello world";
  std::vector<uint8_t> c(4096);
  oracle_iov one = {(const uint8_t*)x, strlen(x)};
  uint32_t n = (uint32_t)oracle_range_compress(&one, 1, strlen(x), c.data(), c.size());
  uint8_t *d_in, *d_out; uint64_t* d_off; uint32_t *d_len, *d_lim, *d_sz; void* d_ar;
  CK(hipMalloc(&d_in, 4096)); CK(hipMalloc(&d_out, 8192)); CK(hipMalloc(&d_off, 8));
  CK(hipMalloc(&d_len, 4)); CK(hipMalloc(&d_lim, 4)); CK(hipMalloc(&d_sz, 4)); CK(hipMalloc(&d_ar, 65536));
  uint64_t off = 0; uint32_t lim = 4000;
  CK(hipMemcpy(d_in, c.data(), n, hipMemcpyHostToDevice));
  CK(hipMemcpy(d_off, &off, 8, hipMemcpyHostToDevice));
  CK(hipMemcpy(d_len, &n, 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(d_lim, &lim, 4, hipMemcpyHostToDevice));
  for (int fill : {0, 0xAB, 0}) {
    for (int dec = 0; dec < 2; ++dec) {
      CK(hipMemset(d_ar, fill, 65536));
      CK(hipMemset(d_out, 0, 8192));
      if (dec) {
        CK(enet_crc::launch_range(true, d_in, d_off, d_len, 1, d_out, d_off, d_lim, d_sz, d_ar, 1, 0));
      } else {
        uint32_t L = (uint32_t)strlen(x);
        CK(hipMemcpy(d_in + 2048, x, L, hipMemcpyHostToDevice));
        uint64_t o2 = 2048;
        uint64_t* d_o2; uint32_t* d_l2; CK(hipMalloc(&d_o2, 8)); CK(hipMalloc(&d_l2, 4));
        CK(hipMemcpy(d_o2, &o2, 8, hipMemcpyHostToDevice)); CK(hipMemcpy(d_l2, &L, 4, hipMemcpyHostToDevice));
        CK(enet_crc::launch_range(false, d_in, d_o2, d_l2, 1, d_out, d_off, d_lim, d_sz, d_ar, 1, 0));
      }
      CK(hipDeviceSynchronize());
      uint32_t sz = 0; char buf[64] = {0};
      CK(hipMemcpy(&sz, d_sz, 4, hipMemcpyDeviceToHost));
      CK(hipMemcpy(buf, d_out, 40, hipMemcpyDeviceToHost));
      if (dec) printf("fill=%02x decompress ret=%u out='%.*s'\n", fill, sz, (int)(sz < 40 ? sz : 40), buf);
      else printf("fill=%02x compress ret=%u match=%d\n", fill, sz, sz == n && memcmp(buf, c.data(), n) == 0);
    }
  }
  return 0;
}
