// crc32_gf2.h -- GF(2) arithmetic for CRC-32/ISO-HDLC (reflected poly 0xEDB88320),
// shared by the host side of libambrycrc and the gfx950 kernels.
//
// Representation: a uint32_t v is a polynomial of degree < 32 in the reflected
// bit order used by Ambry's Crc32 (ambry-utils/.../utils/Crc32.java:154-179) and
// by java.util.zip.CRC32: bit 31 is the coefficient of x^0, bit 0 of x^31.
// In that order, advancing a raw CRC register r over n zero bytes is
//     r  ->  r * x^(8n) mod P          (gf2_mul(r, xpow8(n)))
// and the register after message A||B satisfies
//     R(A||B) = R(A) * x^(8|B|)  xor  R(B)
// which is what lets the kernels split a chunk across lanes, waves and tiles.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#define AMBRY_HD __host__ __device__ __forceinline__
#else
#define AMBRY_HD static inline
#endif

namespace ambrycrc {

constexpr uint32_t kPoly = 0xEDB88320u;  // reflected 0x04C11DB7
constexpr uint32_t kOne = 0x80000000u;   // x^0 in reflected order

// a * b mod P, branch-free (32 shift/xor rounds).
AMBRY_HD uint32_t gf2_mul(uint32_t a, uint32_t b) {
  uint32_t p = 0;
  for (int i = 0; i < 32; ++i) {
    p ^= b & (0u - ((a >> (31 - i)) & 1u));
    b = (b >> 1) ^ (kPoly & (0u - (b & 1u)));
  }
  return p;
}

// x^(8 * 2^k) mod P for k = 0..63, by repeated squaring of x^8.
inline void xpow8_pow2_table(uint32_t out[64]) {
  uint32_t x8 = kOne >> 8;  // x^8
  out[0] = x8;
  for (int k = 1; k < 64; ++k) out[k] = gf2_mul(out[k - 1], out[k - 1]);
}

// x^(8n) mod P (host helper; O(popcount(n)) multiplies).
inline uint32_t xpow8(uint64_t n) {
  uint32_t t[64];
  xpow8_pow2_table(t);
  uint32_t r = kOne;
  for (int k = 0; n; ++k, n >>= 1)
    if (n & 1) r = gf2_mul(r, t[k]);
  return r;
}

// zlib-compatible combine of finalized CRCs: crc(A||B) from crc(A), crc(B), |B|.
inline uint32_t combine(uint32_t crc1, uint32_t crc2, uint64_t len2) {
  return gf2_mul(crc1, xpow8(len2)) ^ crc2;
}

// Byte table T0 (reflected, poly 0xEDB88320) and slice tables T_k = T_{k-1} * x^8.
inline void slice_tables(uint32_t t[][256], int nslices) {
  for (uint32_t i = 0; i < 256; ++i) {
    uint32_t c = i;
    for (int k = 0; k < 8; ++k) c = (c & 1) ? (c >> 1) ^ kPoly : (c >> 1);
    t[0][i] = c;
  }
  for (int k = 1; k < nslices; ++k)
    for (int i = 0; i < 256; ++i) t[k][i] = (t[k - 1][i] >> 8) ^ t[0][t[k - 1][i] & 0xff];
}

// Nibble tables for v -> v * c mod P: N[n][x] = (x << 4n) * c, n = 0..7, x = 0..15,
// so v * c = xor_n N[n][(v >> 4n) & 15]. 16 entries occupy 16 distinct LDS banks,
// so a wave's lookups into one of them never bank-conflict.
inline void nibble_tables(uint32_t c, uint32_t out[8][16]) {
  for (int n = 0; n < 8; ++n)
    for (uint32_t x = 0; x < 16; ++x) out[n][x] = gf2_mul(x << (4 * n), c);
}

}  // namespace ambrycrc
