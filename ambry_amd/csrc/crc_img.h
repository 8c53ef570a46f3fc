// crc_img.h -- device helpers for thread-per-message kernels that hash a few short spans
// (headers, blob record heads) straight from the table image in global memory (L2-resident;
// no LDS staging): T0[b] sits at image byte b << 8 (crc32_layout.h), and the 64 words
// x^(8*2^k) follow the LDS image.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "crc32_gf2.h"
#include "crc32_layout.h"

namespace ambrycrc {

// zlib-style crc32(crc, p[0..n)), one table lookup per byte.
__device__ __forceinline__ uint32_t crc_bytes_img(const uint32_t* __restrict__ img, uint32_t crc,
                                                  const uint8_t* p, uint32_t n) {
  uint32_t c = ~crc;
  for (uint32_t i = 0; i < n; ++i) c = img[((c ^ p[i]) & 0xFFu) << 6] ^ (c >> 8);
  return ~c;
}

// v * x^(8n) mod P: v advanced over n zero bytes (CRC combine; crc32_gf2.h).
__device__ __forceinline__ uint32_t mul_xpow8_img(const uint32_t* __restrict__ img, uint32_t v, uint64_t n) {
  const uint32_t* xp = img + kLdsBytes / 4;
  for (uint32_t k = 0; n; ++k, n >>= 1)
    if (n & 1u) v = gf2_mul(v, xp[k]);
  return v;
}

}  // namespace ambrycrc
