// host_crc.cpp -- host streaming CRC-32 (the CPU side of ambrycrc_update).
//
// Small records (message headers, properties, user metadata, PutRequest fields)
// never cross to the GPU; they are CRC'd here. The reference does this with the
// slice-by-8 loop of Crc32.java:55-98 and, for java.util.zip.CRC32, HotSpot's
// CLMUL intrinsic. This file does the same two things:
//   - slice-by-8 for short inputs (< 64 B) and CPUs without PCLMULQDQ;
//   - a carry-less-multiply fold otherwise: 128-bit lanes of the message are
//     multiplied forward by x^D mod P and xor-ed into the lane D bits later,
//     until one 128-bit remainder is left; its 16 bytes then go through the
//     table from a zero register.
//
// Algebra (same reflected representation as crc32_gf2.h). A 16-byte little-endian
// block is the polynomial X = A*x^64 + B, A = its low qword, B = its high qword,
// with bit j of a qword the coefficient of x^(63-j). PCLMULQDQ of two such
// qwords returns their product times x in the 128-bit frame. Hence
//     X*x^D == clmul(A, x^(64+D-1) mod P) ^ clmul(B, x^(D-1) mod P)   (mod P)
// where a 32-bit reflected constant v sits in the qword as (uint64)v << 32.
// Processing M from register r equals processing M ^ r (r in the first four
// bytes) from zero, so the initial register is xor-ed into the first load.
#include "host_crc.h"

#include <immintrin.h>
#include <stdlib.h>
#include <string.h>

#include "crc32_gf2.h"

namespace ambrycrc {
namespace {

struct Slice8 {
  uint32_t t[8][256];
  Slice8() { slice_tables(t, 8); }
};

const Slice8& s8() {
  static const Slice8 s;
  return s;
}

// Reflected x^m mod P, one multiply by x per step (host init only).
uint32_t xpow_bits(unsigned m) {
  uint32_t r = kOne;
  while (m--) r = (r >> 1) ^ (kPoly & (0u - (r & 1u)));
  return r;
}

// Fold constant pair for distance D bits: qword 0 multiplies A, qword 1 multiplies B.
struct FoldK {
  uint64_t a, b;
};

FoldK fold_k(unsigned d) { return {(uint64_t)xpow_bits(64 + d - 1) << 32, (uint64_t)xpow_bits(d - 1) << 32}; }

struct ClmulConsts {
  FoldK d128, d256, d384, d512, d2048;
  ClmulConsts() : d128(fold_k(128)), d256(fold_k(256)), d384(fold_k(384)), d512(fold_k(512)), d2048(fold_k(2048)) {}
};

const ClmulConsts& kc() {
  static const ClmulConsts c;
  return c;
}

// ------------------------------------------------------------------ SSE PCLMULQDQ
#define AMBRY_SSE_TARGET __attribute__((target("pclmul,sse4.1")))

AMBRY_SSE_TARGET inline __m128i k128(const FoldK& k) { return _mm_set_epi64x((long long)k.b, (long long)k.a); }

AMBRY_SSE_TARGET inline __m128i fold128(__m128i x, __m128i k, __m128i next) {
  const __m128i lo = _mm_clmulepi64_si128(x, k, 0x00);
  const __m128i hi = _mm_clmulepi64_si128(x, k, 0x11);
  return _mm_xor_si128(_mm_xor_si128(lo, hi), next);
}

// The last 128-bit remainder: its CRC from a zero register, then the tail bytes.
AMBRY_SSE_TARGET uint32_t finish(__m128i x, const uint8_t* tail, size_t t) {
  alignas(16) uint8_t buf[16];
  _mm_store_si128(reinterpret_cast<__m128i*>(buf), x);
  return host_update_slice8(host_update_slice8(0u, buf, 16), tail, t);
}

// n >= 64.
AMBRY_SSE_TARGET uint32_t update_pclmul(uint32_t reg, const uint8_t* p, size_t n) {
  const ClmulConsts& c = kc();
  const __m128i* q = reinterpret_cast<const __m128i*>(p);
  __m128i x0 = _mm_xor_si128(_mm_loadu_si128(q + 0), _mm_cvtsi32_si128((int)reg));
  __m128i x1 = _mm_loadu_si128(q + 1), x2 = _mm_loadu_si128(q + 2), x3 = _mm_loadu_si128(q + 3);
  q += 4;
  size_t blocks = n / 16 - 4;
  const __m128i k512 = k128(c.d512);
  for (; blocks >= 4; blocks -= 4, q += 4) {
    x0 = fold128(x0, k512, _mm_loadu_si128(q + 0));
    x1 = fold128(x1, k512, _mm_loadu_si128(q + 1));
    x2 = fold128(x2, k512, _mm_loadu_si128(q + 2));
    x3 = fold128(x3, k512, _mm_loadu_si128(q + 3));
  }
  const __m128i k1 = k128(c.d128);
  __m128i x = fold128(fold128(fold128(x0, k1, x1), k1, x2), k1, x3);
  for (; blocks; --blocks, ++q) x = fold128(x, k1, _mm_loadu_si128(q));
  return finish(x, p + (n & ~size_t(15)), n & 15);
}

// ------------------------------------------------------------ AVX-512 VPCLMULQDQ
#define AMBRY_AVX512_TARGET __attribute__((target("avx512f,avx512bw,vpclmulqdq,pclmul,sse4.1")))

AMBRY_AVX512_TARGET inline __m512i k512x4(const FoldK& k) {
  return _mm512_broadcast_i32x4(_mm_set_epi64x((long long)k.b, (long long)k.a));
}

AMBRY_AVX512_TARGET inline __m512i fold512(__m512i x, __m512i k, __m512i next) {
  const __m512i lo = _mm512_clmulepi64_epi128(x, k, 0x00);
  const __m512i hi = _mm512_clmulepi64_epi128(x, k, 0x11);
  return _mm512_ternarylogic_epi64(lo, hi, next, 0x96);  // lo ^ hi ^ next
}

// n >= 256: four 64-B accumulators, 256 B per iteration.
AMBRY_AVX512_TARGET uint32_t update_vpclmul(uint32_t reg, const uint8_t* p, size_t n) {
  const ClmulConsts& c = kc();
  const uint8_t* q = p;
  __m512i z0 = _mm512_xor_si512(_mm512_loadu_si512(q), _mm512_castsi128_si512(_mm_cvtsi32_si128((int)reg)));
  __m512i z1 = _mm512_loadu_si512(q + 64), z2 = _mm512_loadu_si512(q + 128), z3 = _mm512_loadu_si512(q + 192);
  q += 256;
  size_t rem = n - 256;
  const __m512i k2048 = k512x4(c.d2048);
  for (; rem >= 256; rem -= 256, q += 256) {
    z0 = fold512(z0, k2048, _mm512_loadu_si512(q));
    z1 = fold512(z1, k2048, _mm512_loadu_si512(q + 64));
    z2 = fold512(z2, k2048, _mm512_loadu_si512(q + 128));
    z3 = fold512(z3, k2048, _mm512_loadu_si512(q + 192));
  }
  const __m512i k4 = k512x4(c.d512);
  __m512i z = fold512(fold512(fold512(z0, k4, z1), k4, z2), k4, z3);
  for (; rem >= 64; rem -= 64, q += 64) z = fold512(z, k4, _mm512_loadu_si512(q));
  // Four 128-bit lanes at distances 384, 256, 128, 0 from the end of the last one.
  const __m128i l0 = _mm512_extracti32x4_epi32(z, 0), l1 = _mm512_extracti32x4_epi32(z, 1);
  const __m128i l2 = _mm512_extracti32x4_epi32(z, 2), l3 = _mm512_extracti32x4_epi32(z, 3);
  __m128i x = _mm_xor_si128(fold128(l0, k128(c.d384), l3), fold128(l1, k128(c.d256), _mm_setzero_si128()));
  x = fold128(l2, k128(c.d128), x);
  const __m128i k1 = k128(c.d128);
  for (; rem >= 16; rem -= 16, q += 16) x = fold128(x, k1, _mm_loadu_si128(reinterpret_cast<const __m128i*>(q)));
  return finish(x, q, rem);
}

int select_impl() {
  int best = kHostSlice8;
  __builtin_cpu_init();
  if (__builtin_cpu_supports("pclmul") && __builtin_cpu_supports("sse4.1")) best = kHostPclmul;
  if (best == kHostPclmul && __builtin_cpu_supports("avx512f") && __builtin_cpu_supports("avx512bw") &&
      __builtin_cpu_supports("vpclmulqdq"))
    best = kHostVpclmul;
  const char* e = getenv("AMBRYCRC_HOST_IMPL");
  if (e) {
    for (int i = 0; i <= best; ++i)
      if (strcmp(e, host_impl_name(i)) == 0) return i;  // cannot force an unsupported one
  }
  return best;
}

}  // namespace

uint32_t host_update_slice8(uint32_t c, const uint8_t* p, size_t n) {
  const Slice8& h = s8();
  while (n >= 8) {
    uint32_t lo, hi;
    memcpy(&lo, p, 4);
    memcpy(&hi, p + 4, 4);
    lo ^= c;
    c = h.t[7][lo & 0xff] ^ h.t[6][(lo >> 8) & 0xff] ^ h.t[5][(lo >> 16) & 0xff] ^ h.t[4][lo >> 24] ^
        h.t[3][hi & 0xff] ^ h.t[2][(hi >> 8) & 0xff] ^ h.t[1][(hi >> 16) & 0xff] ^ h.t[0][hi >> 24];
    p += 8;
    n -= 8;
  }
  while (n--) c = (c >> 8) ^ h.t[0][(c ^ *p++) & 0xff];
  return c;
}

int host_impl() {
  static const int impl = select_impl();
  return impl;
}

const char* host_impl_name(int impl) {
  switch (impl) {
    case kHostSlice8: return "slice8";
    case kHostPclmul: return "pclmul";
    case kHostVpclmul: return "vpclmul";
    default: return "unknown";
  }
}

uint32_t host_update_reg(uint32_t reg, const uint8_t* p, size_t n) {
  const int impl = host_impl();
  if (impl == kHostVpclmul && n >= 256) return update_vpclmul(reg, p, n);
  if (impl >= kHostPclmul && n >= 64) return update_pclmul(reg, p, n);
  return host_update_slice8(reg, p, n);
}

}  // namespace ambrycrc
