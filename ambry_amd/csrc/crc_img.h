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

// Slice-by-4 tables T0..T3 (T_j[b] = b advanced over j further zero bytes), 4 KiB, staged
// into LDS per workgroup from the table image: T_j[b] sits at image byte
// (j>>1)<<16 | b<<8 | (j&1)<<7 (lane column 0), crc32_layout.h; t[256j + b] = T_j[b].
// 256-thread blocks: each thread issues its 4 loads before its 4 LDS stores (one memory
// round trip, not four).
__device__ __forceinline__ void stage_slice_tables(uint32_t* __restrict__ t, const uint32_t* __restrict__ img) {
  uint32_t v[4];
#pragma unroll
  for (uint32_t r = 0; r < 4; ++r) {
    const uint32_t i = threadIdx.x + 256u * r, j = i >> 8, b = i & 255u;
    v[r] = img[(((j >> 1) << 16) | (b << 8) | ((j & 1) << 7)) >> 2];
  }
#pragma unroll
  for (uint32_t r = 0; r < 4; ++r) t[threadIdx.x + 256u * r] = v[r];
}

// crc32(crc, b[0..n)) of n <= N bytes held in registers, through the LDS tables of
// stage_slice_tables: slice-by-4 over whole words, then bytes.
template <int N>
__device__ __forceinline__ uint32_t crc_regs_lds(const uint32_t* __restrict__ t, uint32_t crc, const uint8_t (&b)[N],
                                                 uint32_t n) {
  uint32_t c = ~crc;
#pragma unroll
  for (int w = 0; w < N / 4; ++w) {
    if ((uint32_t)(4 * w + 4) <= n) {
      const uint32_t x = c ^ ((uint32_t)b[4 * w] | (uint32_t)b[4 * w + 1] << 8 | (uint32_t)b[4 * w + 2] << 16 |
                              (uint32_t)b[4 * w + 3] << 24);
      c = t[768 + (x & 0xffu)] ^ t[512 + ((x >> 8) & 0xffu)] ^ t[256 + ((x >> 16) & 0xffu)] ^ t[x >> 24];
    }
  }
  const uint32_t done = n & ~3u;
#pragma unroll
  for (int i = 0; i < N; ++i)
    if ((uint32_t)i >= done && (uint32_t)i < n) c = t[(c ^ b[i]) & 0xffu] ^ (c >> 8);
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
