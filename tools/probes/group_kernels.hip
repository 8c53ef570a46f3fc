// group_kernels.hip -- the high-occupancy group kernel (variant 32): whole small chunks
// (1 B .. kGroupSmallMax) of a batch, outside the fused sweep kernel.
//
// Why a kernel of its own: the fused kernel's group phase is latency-bound at the
// 16 waves per CU its 149.5 KiB LDS image and 128 VGPRs allow (8 / 12 / 16 waves measured
// 433 / 341 / 304 us on 4 KiB-blob messages). Here the image is 72.5 KiB and a lane holds at most
// 64 VGPRs, so two 1024-thread workgroups share a CU: 32 waves, twice the bytes in flight.
//
//   LDS image  [0, 64 KiB): T0, T1 of the main image (crc32_layout.h: byte b at address bits
//              8..15, table at bit 7, lane column at bits 2..6 -- 32 copies, conflict-free
//              ds_read_b32); [64 KiB, +8.5 KiB): the main image's nibble sets FOLD, TREE[0..5],
//              POW[0..9]. No T2/T3: the chain is slice-by-2 (two dependent table steps per
//              4 bytes instead of one; 32 waves hide the longer chain, the lookups per byte are
//              the same and stay conflict-free).
//   classes    as the fused phase's: class 0 (<= 256 B) in G0-lane groups of 16-B pieces
//              (fold x^(8*16 G0) per piece); classes 1 (<= 1 KiB), 2 (<= 4 KiB), 3 (<= 16 KiB)
//              in 8-, 16-, 16-lane groups of 64-B lane runs (4 coalesced loads per lane, quad
//              transpose, fold x^(8*64G) per super-block). Rounds are not streamed across chunk
//              boundaries: with 32 waves per CU the other waves cover a round's descriptor trips.
//   per chunk  the initial register ~crc_in is XORed into the chunk's first 4 bytes, the group's
//              lane states merge by a log2(G)-level nibble tree, the < 16 trailing bytes go
//              16/G per lane, xor-out; the group leader stores out[chunk] (and exp_fill / the
//              copy-through bytes as the fused phase does).
#ifndef AMBRY_AB_SPLIT_GROUP
#error "A/B only: tools/ab_build.sh builds it with -DAMBRY_AB_SPLIT_GROUP -DAMBRY_AB_PROBE_BUILD"
#endif
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "crc32_gf2.h"
#include "crc32_kernels.h"
#include "crc32_layout.h"

namespace ambrycrc {
namespace g2 {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) u32x4 gu32x4;
typedef __attribute__((address_space(1))) uint8_t gu8;

constexpr uint32_t kSlice2Bytes = 64u * 1024u;                       // T0, T1 x 32 lane copies
constexpr uint32_t kNibArea = kPowOff + 10u * kNibSetBytes;          // FOLD, TREE[0..5], POW[0..9]
constexpr uint32_t kImgBytes = kSlice2Bytes + kNibArea;              // 72.5 KiB
static_assert(kImgBytes <= 80u * 1024u, "two workgroups per CU");

__shared__ __attribute__((aligned(16))) uint32_t lds[kImgBytes / 4];

__device__ __forceinline__ uint32_t rd(uint32_t byte_addr) {
  return *reinterpret_cast<const uint32_t*>(reinterpret_cast<const char*>(lds) + byte_addr);
}

// LDS-DMA staging (global_load_lds_dwordx4, 1 KiB per wave instruction): image bytes [0, 64 KiB)
// and [kSliceBytes, kSliceBytes + kNibArea).
__device__ __forceinline__ void fill(const uint32_t* __restrict__ img) {
  const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
  constexpr uint32_t kChunks = (kImgBytes + 1023) / 1024;
  for (uint32_t c = wave; c < kChunks; c += nw) {
    const uint32_t dst = c * 1024 + lane * 16;
    const uint32_t src = dst < kSlice2Bytes ? dst : dst - kSlice2Bytes + kSliceBytes;
    if (dst < kImgBytes)
      __builtin_amdgcn_global_load_lds(
          (const __attribute__((address_space(1))) void*)(reinterpret_cast<const uint8_t*>(img) + src),
          (__attribute__((address_space(3))) void*)(reinterpret_cast<uint8_t*>(lds) + c * 1024), 16, 0, 0);
  }
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();
}

__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}

template <int CTRL, int ROWS>
__device__ __forceinline__ uint32_t dpp(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, ROWS, 0xf, false);
}
template <int CTRL>
__device__ __forceinline__ uint32_t dppq(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, CTRL, 0xf, 0xf, true);
}

// v * C mod P, C's nibble tables at nib area offset set_off (8 conflict-free lookups).
__device__ __forceinline__ uint32_t nib_mul(uint32_t v, uint32_t set_off) {
  uint32_t t[8];
#pragma unroll
  for (int n = 0; n < 8; ++n) t[n] = rd(kSlice2Bytes + set_off + 64u * n + (__builtin_amdgcn_ubfe(v, 4 * n, 4) << 2));
  return xor3(xor3(t[0], t[1], t[2]), xor3(t[3], t[4], t[5]), t[6] ^ t[7]);
}
__device__ __forceinline__ uint32_t pow_mul(uint32_t v, uint32_t k) { return nib_mul(v, kPowOff + kNibSetBytes * k); }

// Lane constants: L0 = T0's lane column, L1 = T1's (bit 7). v_perm builds an entry address
// from one of them and a byte of the state (byte 1 of the result = that byte).
struct Lane2 {
  uint32_t L0, L1;
};
__device__ __forceinline__ Lane2 lane2(uint32_t lane) {
  const uint32_t col = (lane & 31u) << 2;
  return Lane2{col, (1u << 7) | col};
}

// Two bytes of the raw chain: T1[x.b0] ^ T0[x.b1] ^ (x >> 16) (slice-by-2, a5's T8_0/T8_1).
__device__ __forceinline__ uint32_t s2(uint32_t x, const Lane2& k) {
  const uint32_t a1 = __builtin_amdgcn_perm(k.L1, x, 0x0C060004u);
  const uint32_t a0 = __builtin_amdgcn_perm(k.L0, x, 0x0C060104u);
  return xor3(rd(a1), rd(a0), x >> 16);
}
// Four bytes, xor the next word: slice-by-4 as two slice-by-2 steps.
__device__ __forceinline__ uint32_t s4(uint32_t x, const Lane2& k, uint32_t xin) { return s2(s2(x, k), k) ^ xin; }

// Raw CRC (zero register) of R consecutive 16-B pieces, xor xin into the last step.
template <int R>
__device__ __forceinline__ uint32_t run_crc(const u32x4 (&w)[R], const Lane2& k, uint32_t xin) {
  uint32_t x = w[0].x;
#pragma unroll
  for (int r = 0; r < R; ++r) {
    x = s4(x, k, w[r].y);
    x = s4(x, k, w[r].z);
    x = s4(x, k, w[r].w);
    x = s4(x, k, r + 1 < R ? w[r + 1].x : xin);
  }
  return x;
}

// T0[b] advanced over kk further zero bytes (kk < 16), from T0/T1 and POW[1..3].
__device__ __forceinline__ uint32_t byte_at(uint32_t b, uint32_t kk, uint32_t lane) {
  uint32_t v = rd((b << 8) | ((kk & 1u) << 7) | ((lane & 31u) << 2));
  if (kk & 2u) v = pow_mul(v, 1);
  if (kk & 4u) v = pow_mul(v, 2);
  if (kk & 8u) v = pow_mul(v, 3);
  return v;
}

// 4x4 transpose of 16-B elements inside each lane quad (crc32_kernels.hip quad_transpose_asm).
__device__ __forceinline__ void quad_transpose(u32x4 (&x)[4]) {
  const uint64_t m1 = 0xAAAAAAAAAAAAAAAAull, n1 = 0x5555555555555555ull;
  const uint64_t m2 = 0xCCCCCCCCCCCCCCCCull, n2 = 0x3333333333333333ull;
#pragma unroll
  for (int d = 0; d < 4; ++d) {
    uint32_t a0, a1, a2, a3, y0, y1, y2, y3;
    asm volatile(
        "s_nop 1\n\t"
        "s_mov_b64 vcc, %[n1]\n\t"
        "v_cndmask_b32_dpp %[a0], %[x1], %[x0], vcc quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
        "v_cndmask_b32_dpp %[a2], %[x3], %[x2], vcc quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
        "s_mov_b64 vcc, %[m1]\n\t"
        "v_cndmask_b32_dpp %[a1], %[x0], %[x1], vcc quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
        "v_cndmask_b32_dpp %[a3], %[x2], %[x3], vcc quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
        "s_mov_b64 vcc, %[n2]\n\t"
        "v_cndmask_b32_dpp %[y0], %[a2], %[a0], vcc quad_perm:[2,3,0,1] row_mask:0xf bank_mask:0xf\n\t"
        "v_cndmask_b32_dpp %[y1], %[a3], %[a1], vcc quad_perm:[2,3,0,1] row_mask:0xf bank_mask:0xf\n\t"
        "s_mov_b64 vcc, %[m2]\n\t"
        "v_cndmask_b32_dpp %[y2], %[a0], %[a2], vcc quad_perm:[2,3,0,1] row_mask:0xf bank_mask:0xf\n\t"
        "v_cndmask_b32_dpp %[y3], %[a1], %[a3], vcc quad_perm:[2,3,0,1] row_mask:0xf bank_mask:0xf\n\t"
        "s_nop 1"
        : [a0] "=&v"(a0), [a1] "=&v"(a1), [a2] "=&v"(a2), [a3] "=&v"(a3), [y0] "=&v"(y0), [y1] "=&v"(y1),
          [y2] "=&v"(y2), [y3] "=&v"(y3)
        : [x0] "v"(x[0][d]), [x1] "v"(x[1][d]), [x2] "v"(x[2][d]), [x3] "v"(x[3][d]), [m1] "s"(m1), [n1] "s"(n1),
          [m2] "s"(m2), [n2] "s"(n2)
        : "vcc");
    x[0][d] = y0;
    x[1][d] = y1;
    x[2][d] = y2;
    x[3][d] = y3;
  }
}

// Lane-bit tree level: lanes with bit BIT set absorb the partner's state shifted by POW[POWK].
template <int BIT, int POWK>
__device__ __forceinline__ uint32_t tree_level(uint32_t s, uint32_t lane) {
  uint32_t o;
  if constexpr (BIT == 0) o = dpp<0x111, 0xf>(s);       // row_shr:1
  else if constexpr (BIT == 1) o = dpp<0x112, 0xf>(s);  // row_shr:2
  else if constexpr (BIT == 2) o = dpp<0x114, 0xf>(s);  // row_shr:4
  else o = dpp<0x118, 0xf>(s);                          // row_shr:8
  const uint32_t sh = pow_mul(o, POWK);
  return (lane & (1u << BIT)) ? (s ^ sh) : s;
}

// xor over the G lanes of each group; result in every lane of the group
template <int G>
__device__ __forceinline__ uint32_t group_xor(uint32_t v) {
  if constexpr (G == 16) {
    v ^= dpp<0x128, 0xf>(v);
    v ^= dpp<0x124, 0xf>(v);
    v ^= dpp<0x122, 0xf>(v);
    v ^= dpp<0x121, 0xf>(v);
  } else {
    static_assert(G == 2 || G == 4 || G == 8, "group width");
    v ^= dppq<0xB1>(v);
    if constexpr (G >= 4) v ^= dppq<0x4E>(v);
    if constexpr (G == 8) v ^= (uint32_t)__shfl_xor((int)v, 4);
  }
  return v;
}

__device__ __forceinline__ uint64_t aligned_end(uint64_t s, uint64_t e) {
  const uint64_t b = e & ~uint64_t(15);
  return b < s ? s : b;
}

// XOR the initial register (little-endian bytes at [cs, cs+4)) into the piece at p and zero the
// bytes before cs (a piece entirely before cs was loaded from the dummy address: zero it).
__device__ __forceinline__ void fix_piece(u32x4& w, int64_t p, uint64_t cs, uint32_t rinit) {
  if (p + 16 <= (int64_t)cs) w = u32x4{0u, 0u, 0u, 0u};
  if (p < (int64_t)cs + 4 && p + 16 > (int64_t)cs) {
    const int64_t o = (int64_t)cs - p;
#pragma unroll
    for (int d = 0; d < 4; ++d) {
      const int64_t od = o - 4 * d;
      if (od >= 0 && od < 4) w[d] ^= rinit << (8 * (uint32_t)od);
      else if (od < 0 && od > -4) w[d] ^= rinit >> (8 * (uint32_t)(-od));
    }
    if (p < (int64_t)cs) {
      const uint32_t cut = (uint32_t)((int64_t)cs - p);
#pragma unroll
      for (int d = 0; d < 4; ++d) {
        const int lo = (int)cut - 4 * d;
        const uint32_t m = lo <= 0 ? 0xFFFFFFFFu : (lo >= 4 ? 0u : (0xFFFFFFFFu << (8 * lo)));
        w[d] &= m;
      }
    }
  }
}

__device__ __forceinline__ void st8g(uint8_t* d, uint32_t v) { *(gu8*)d = (uint8_t)v; }
// copy-through of a piece loaded at source offset p: the bytes from lo on go to dbase + p
__device__ __forceinline__ void copy_piece(uint8_t* dbase, int64_t p, const u32x4& v, int64_t lo) {
  if (!dbase || p + 16 <= lo) return;
  if (p >= lo) {
    *(gu32x4*)(dbase + p) = v;
    return;
  }
#pragma unroll
  for (int b = 0; b < 16; ++b)
    if (p + b >= lo) st8g(dbase + p + b, v[b >> 2] >> (8 * (b & 3)));
}

template <int G>
__device__ __forceinline__ uint64_t group_per(uint64_t ns, uint64_t nwaves) {
  return ((ns + nwaves - 1) / nwaves + 64 / G - 1) / (64 / G) * (64 / G);
}

// One round's chunk (per lane: its group's chunk). Loads whose piece lies outside the chunk
// read 16 B of the table image (`dummy`, cache-resident) and are zeroed after: every load is
// issued unconditionally, so the count in flight never depends on the path.
struct Chunk {
  uint64_t cs, cb;
  uint32_t t;      // trailing bytes (< 16) after cb
  uint32_t rinit;  // ~crc_in
  uint32_t ci;
  bool act;
};

template <int G>
__device__ __forceinline__ Chunk load_chunk(const SweepArgs& a, uint64_t i, uint64_t i1, uint32_t gi) {
  Chunk c;
  c.act = i + gi < i1;
  c.ci = c.act ? a.small_idx[i + gi] : 0u;
  const uint64_t len = c.act ? a.len[c.ci] : 0;
  c.cs = c.act ? a.off[c.ci] : 0;
  c.rinit = ~(c.act && a.crc_in ? a.crc_in[c.ci] : 0u);
  const uint64_t ce = c.cs + len;
  c.cb = aligned_end(c.cs, ce);
  c.t = (uint32_t)(ce - c.cb);
  return c;
}

// Wave maximum of a group-uniform value (one readlane per group).
template <int G>
__device__ __forceinline__ uint32_t wave_max(uint32_t v) {
  uint32_t m = 0;
#pragma unroll
  for (uint32_t q = 0; q < 64 / G; ++q) {
    const uint32_t x = __builtin_amdgcn_readlane(v, q * G);
    m = x > m ? x : m;
  }
  return m;
}

// The chunk's CRC from the group's merged body register r (valid in every lane of the group):
// shift over the t trailing bytes, add theirs (16/G per lane: lane gl has the bytes at distance
// kk in [k0, k0 + 16/G) from the end, T0[b] * x^(8 kk)), xor-out, short-chunk init term.
template <int G>
__device__ __forceinline__ uint32_t finish(const SweepArgs& a, const uint8_t* __restrict__ dummy, const Chunk& c,
                                           uint32_t r, uint32_t lane, uint8_t* dsh) {
  constexpr uint32_t BPL = 16u / G;
  constexpr uint32_t NP = (BPL + 1) / 2;  // byte pairs per lane
  const uint32_t k0 = BPL * (G - 1 - (lane & (G - 1)));
  const uint64_t ce = c.cb + c.t;
  uint32_t tb[BPL];  // issued before the shifts below; bytes past t read as 0 (T0[0] = 0)
#pragma unroll
  for (uint32_t i = 0; i < BPL; ++i) tb[i] = k0 + i < c.t ? a.base[ce - 1 - (k0 + i)] : 0u;
  if (c.t & 1u) r = pow_mul(r, 0);
  if (c.t & 2u) r = pow_mul(r, 1);
  if (c.t & 4u) r = pow_mul(r, 2);
  if (c.t & 8u) r = pow_mul(r, 3);
  uint32_t v = 0;
  if (k0 < c.t) {
#pragma unroll
    for (uint32_t i = 0; i < BPL; ++i) {
      const uint32_t kk = k0 + i;
      if (kk < c.t) {
        const uint64_t at = ce - 1 - kk;
        if (dsh) st8g(dsh + at, tb[i]);
        if (at < c.cs + 4) tb[i] ^= (c.rinit >> (8 * (uint32_t)(at - c.cs))) & 0xFFu;
      }
    }
    if constexpr (BPL == 1) {
      v = byte_at(tb[0], k0, lane);
    } else {  // pairs from the farthest: v = v * x^16 ^ T0[b(k0+2h)] ^ T1[b(k0+2h+1)], then * x^(8 k0)
#pragma unroll
      for (int h = (int)NP - 1; h >= 0; --h) {
        if (h != (int)NP - 1) v = pow_mul(v, 1);
        v ^= rd((tb[2 * h] << 8) | ((lane & 31u) << 2));
        if (2 * h + 1 < (int)BPL) v ^= rd((tb[2 * h + 1] << 8) | (1u << 7) | ((lane & 31u) << 2));
      }
      if (k0 & 2u) v = pow_mul(v, 1);
      if (k0 & 4u) v = pow_mul(v, 2);
      if (k0 & 8u) v = pow_mul(v, 3);
    }
  }
  v = group_xor<G>(v);
  uint32_t crc = r ^ v ^ 0xFFFFFFFFu;
  const uint64_t len = ce - c.cs;
  if (len < 4) crc ^= c.rinit >> (8 * (uint32_t)len);
  return crc;
}

template <int G>
__device__ __forceinline__ void store(const SweepArgs& a, const Chunk& c, uint32_t crc, uint64_t stored,
                                      uint32_t lane) {
  if ((lane & (G - 1)) == 0 && c.act) {
    a.out[c.ci] = crc;
    if (a.exp_fill) {
      const uint64_t st = __builtin_bswap64(stored);
      a.exp_fill[c.ci] = (st >> 32) ? ~crc : (uint32_t)st;
    }
  }
}

// message verify: the record's stored CRC follows its bytes (leader lane; others read the dummy)
template <int G>
__device__ __forceinline__ uint64_t load_stored(const SweepArgs& a, const uint8_t* __restrict__ dummy,
                                                const Chunk& c, uint32_t lane) {
  uint64_t stored = 0;
  if (a.exp_fill) {
    const bool leader = (lane & (G - 1)) == 0 && c.act;
    __builtin_memcpy(&stored, leader ? a.base + c.cb + c.t : dummy, 8);
  }
  return stored;
}

// ---- classes 1-3: 64-B lane runs (G = 8 or 16), one super-block of 64G B per group per step
template <int G, bool COPY>
__device__ __forceinline__ void class_runs(const SweepArgs& a, uint64_t lo, uint64_t hi, uint32_t wave,
                                           uint64_t nwaves, uint32_t lane, const Lane2& k) {
  constexpr uint32_t S = 64 / G;
  constexpr uint32_t SB = 64 * G;  // super-block bytes per group
  constexpr uint32_t kFold = G == 16 ? kFoldOff : kPowOff + kNibSetBytes * 9;  // x^(8*64G)
  constexpr uint32_t LB = G == 8 ? 7u : 8u;                                      // log2(16G)
  if (hi <= lo) return;
  const uint64_t per = group_per<G>(hi - lo, nwaves);
  const uint64_t i0 = lo + (uint64_t)wave * per;
  if (i0 >= hi) return;
  const uint64_t i1 = i0 + per < hi ? i0 + per : hi;
  const uint32_t gi = lane / G;
  const uint8_t* dummy = reinterpret_cast<const uint8_t*>(a.img);
  const int64_t lane_off = 16 * (int64_t)(lane & (G - 1));
#pragma unroll 1
  for (uint64_t i = i0; i < i1; i += S) {
    const Chunk c = load_chunk<G>(a, i, i1, gi);
    uint8_t* dsh = nullptr;
    if constexpr (COPY) {
      const uint64_t co = c.act ? a.copy_off[c.ci] : kCopySkip;
      dsh = co == kCopySkip ? nullptr : a.copy_dst + co - c.cs;
    }
    const uint32_t nbw = wave_max<G>((uint32_t)((c.cb - c.cs + SB - 1) / SB));
    const int64_t p0 = (int64_t)c.cb - (int64_t)nbw * SB + lane_off;
    const uint64_t stored = load_stored<G>(a, dummy, c, lane);
    auto load = [&](uint32_t sb, u32x4 (&x)[4]) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int64_t p = p0 + (int64_t)sb * SB + (16 * G) * q;
        const bool in = sb < nbw && p + 16 > (int64_t)c.cs;  // => floor16(cs) <= p < cb
        x[q] = *reinterpret_cast<const u32x4*>(in ? a.base + p : dummy);
      }
    };
    uint32_t s = 0;
    u32x4 x[4];
    load(0, x);
#pragma unroll 1
    for (uint32_t sb = 0; sb < nbw; ++sb) {
      u32x4 nx[4];
      load(sb + 1, nx);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int64_t p = p0 + (int64_t)sb * SB + (16 * G) * q;
        if constexpr (COPY) copy_piece(dsh, p, x[q], (int64_t)c.cs);
        fix_piece(x[q], p, c.cs, c.rinit);
      }
      quad_transpose(x);
      s = run_crc<4>(x, k, sb ? nib_mul(s, kFold) : 0u);
#pragma unroll
      for (int q = 0; q < 4; ++q) x[q] = nx[q];
    }
    uint32_t r = 0;
    if (nbw) {  // lanes gl = 4m + j: bits 2.. merge the runs of a block, bits 0, 1 the blocks
      r = tree_level<2, 6>(s, lane);
      if constexpr (G == 16) r = tree_level<3, 7>(r, lane);
      r = tree_level<0, LB>(r, lane);
      r = tree_level<1, LB + 1>(r, lane);
    }
    r = __shfl(r, (int)(lane | (G - 1)));
    store<G>(a, c, finish<G>(a, dummy, c, r, lane, dsh), stored, lane);
  }
}

// ---- class 0: G-lane groups of 16-B pieces, lane gl owns [16gl, 16gl + 16) of every 16G-B block
template <int G, bool COPY>
__device__ __forceinline__ void class_pieces(const SweepArgs& a, uint64_t lo, uint64_t hi, uint32_t wave,
                                             uint64_t nwaves, uint32_t lane, const Lane2& k) {
  constexpr uint32_t S = 64 / G;
  constexpr uint32_t BB = 16 * G;
  constexpr uint32_t P = 4;  // pieces in flight per lane
  constexpr uint32_t kFold = kPowOff + kNibSetBytes * (G == 2 ? 5u : G == 4 ? 6u : 7u);  // x^(8*16G)
  if (hi <= lo) return;
  const uint64_t per = group_per<G>(hi - lo, nwaves);
  const uint64_t i0 = lo + (uint64_t)wave * per;
  if (i0 >= hi) return;
  const uint64_t i1 = i0 + per < hi ? i0 + per : hi;
  const uint32_t gi = lane / G;
  const uint8_t* dummy = reinterpret_cast<const uint8_t*>(a.img);
  const int64_t lane_off = 16 * (int64_t)(lane & (G - 1));
#pragma unroll 1
  for (uint64_t i = i0; i < i1; i += S) {
    const Chunk c = load_chunk<G>(a, i, i1, gi);
    uint8_t* dsh = nullptr;
    if constexpr (COPY) {
      const uint64_t co = c.act ? a.copy_off[c.ci] : kCopySkip;
      dsh = co == kCopySkip ? nullptr : a.copy_dst + co - c.cs;
    }
    const uint32_t nbw = wave_max<G>((uint32_t)((c.cb - c.cs + BB - 1) / BB));
    const int64_t p0 = (int64_t)c.cb - (int64_t)nbw * BB + lane_off;
    const uint64_t stored = load_stored<G>(a, dummy, c, lane);
    auto load = [&](uint32_t b) -> u32x4 {
      const int64_t p = p0 + (int64_t)b * BB;
      const bool in = b < nbw && p + 16 > (int64_t)c.cs;
      return *reinterpret_cast<const u32x4*>(in ? a.base + p : dummy);
    };
    u32x4 ring[P];
#pragma unroll
    for (uint32_t u = 0; u < P; ++u) ring[u] = load(u);
    uint32_t s = 0;
#pragma unroll 1
    for (uint32_t b0 = 0; b0 < nbw; b0 += P) {
#pragma unroll
      for (uint32_t u = 0; u < P; ++u) {
        const uint32_t b = b0 + u;
        if (b < nbw) {  // wave-uniform
          u32x4 x = ring[u];
          ring[u] = load(b + P);
          const int64_t p = p0 + (int64_t)b * BB;
          if constexpr (COPY) copy_piece(dsh, p, x, (int64_t)c.cs);
          fix_piece(x, p, c.cs, c.rinit);
          const u32x4 w1[1] = {x};
          s = run_crc<1>(w1, k, b ? nib_mul(s, kFold) : 0u);
        }
      }
    }
    uint32_t r = s;
    if (nbw) {
      r = tree_level<0, 4>(r, lane);  // 16 B
      if constexpr (G >= 4) r = tree_level<1, 5>(r, lane);
      if constexpr (G >= 8) r = tree_level<2, 6>(r, lane);
    }
    r = __shfl(r, (int)(lane | (G - 1)));
    store<G>(a, c, finish<G>(a, dummy, c, r, lane, dsh), stored, lane);
  }
}

#ifndef AMBRY_G2_C0_G
#define AMBRY_G2_C0_G 2
#endif
// occupancy knobs (tools/ab_build.sh AB_FLAGS): waves per SIMD the register budget is sized for,
// threads per workgroup, workgroups launched per CU
#ifndef AMBRY_G2_WPE
#define AMBRY_G2_WPE 8
#endif
#ifndef AMBRY_G2_BLOCK
#define AMBRY_G2_BLOCK 1024
#endif
#ifndef AMBRY_G2_WG_PER_CU
#define AMBRY_G2_WG_PER_CU 2
#endif

// Persistent: wave w takes its share of each class of the plan's small-chunk list
// (small_total = {total, start of class 1, 2, 3}).
template <bool COPY>
__global__ __launch_bounds__(AMBRY_G2_BLOCK) __attribute__((amdgpu_waves_per_eu(AMBRY_G2_WPE))) void crc32_group_kernel(SweepArgs a) {
  const uint64_t c4 = a.small_total[0];
  if (c4 == 0) return;  // uniform
  fill(a.img);
  const uint32_t lane = threadIdx.x & 63u;
  const uint64_t nwaves = (uint64_t)gridDim.x * (blockDim.x >> 6);
  const uint32_t wave = __builtin_amdgcn_readfirstlane((threadIdx.x >> 6) * gridDim.x + blockIdx.x);
  const Lane2 k = lane2(lane);
  const uint64_t c1 = a.small_total[1], c2 = a.small_total[2], c3 = a.small_total[3];
#ifndef AMBRY_G2_ONLY
#define AMBRY_G2_ONLY 15
#endif
  if (AMBRY_G2_ONLY & 1) class_pieces<AMBRY_G2_C0_G, COPY>(a, 0, c1, wave, nwaves, lane, k);
  if (AMBRY_G2_ONLY & 2) class_runs<8, COPY>(a, c1, c2, wave, nwaves, lane, k);
  if (AMBRY_G2_ONLY & 4) class_runs<16, COPY>(a, c2, c3, wave, nwaves, lane, k);
  if (AMBRY_G2_ONLY & 8) class_runs<16, COPY>(a, c3, c4, wave, nwaves, lane, k);
}

}  // namespace g2

hipError_t launch_group(const SweepArgs& a, int num_cu, hipStream_t s) {
  const dim3 grid(num_cu * AMBRY_G2_WG_PER_CU), block(AMBRY_G2_BLOCK);
  if (a.copy_dst) hipLaunchKernelGGL(g2::crc32_group_kernel<true>, grid, block, 0, s, a);
  else hipLaunchKernelGGL(g2::crc32_group_kernel<false>, grid, block, 0, s, a);
  return hipGetLastError();
}

}  // namespace ambrycrc
