// Host CRC loops (ambry_amd/csrc/host_crc.cpp) under AddressSanitizer + UBSan, against zlib:
// every length 0..2999 at three misalignments, each buffer allocated to its exact size so a
// SIMD load past the end is caught. Built and run by tests/test_abi.py (host code only).
#include <zlib.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include "host_crc.h"
int main() {
  int bad = 0;
  for (size_t n = 0; n < 3000; ++n) {
    for (int shift = 0; shift < 3; ++shift) {
      unsigned char* raw = (unsigned char*)malloc(n + shift + 1);
      unsigned char* p = raw + shift;
      for (size_t i = 0; i < n; ++i) p[i] = (unsigned char)(i * 131 + n + shift);
      uint32_t want = (uint32_t)crc32(0x12345678u, p, (uInt)n);
      uint32_t got = ~ambrycrc::host_update_reg(~0x12345678u, p, n);
      if (got != want) ++bad;
      free(raw);
    }
  }
  printf("impl=%s bad=%d\n", ambrycrc::host_impl_name(ambrycrc::host_impl()), bad);
  return bad != 0;
}
