// region_crc.h -- region mode of the message verify, pass 2: a record's CRC assembled from the
// 64-B run sums of pass 1 (region_runs_kernel, crc32_kernels.hip), for the fused per-message
// kernel region_msg_kernel (message_kernels.hip).
//
// Why: a region of small PUT messages read as CRC jobs puts every record through
// the batch engine's group phase, where each record pays a round of descriptors, chain and tree
// (4 KiB-blob messages: 4.5 TB/s). Read as contiguous memory the region streams at the C3 wave
// body's rate; what is left per record is arithmetic on run sums, and re-reading the at most
// two runs its ends cut.
//
// A record = [pa, pb) (offsets from RegionArgs::base), zlib CRC-32 out:
//   runs     A0 = pa rounded down, B1 = pb rounded up to 64 B: n = (B1 - A0) / 64 runs, run r at
//            A0 + 64r. Every value below is a raw CRC register "at the end of its run".
//   head     run 0 from the bytes: bytes outside [pa, pb) zeroed (leading zeros leave a zero
//            register unchanged; trailing ones advance it to the run end), the initial register
//            ~0 XORed into the first four record bytes (when the run holds t < 4 of them, the
//            rest of the register, ~0 >> 8t, is added at the run end).
//   tail     run n-1 from the bytes (bytes from pb on zeroed) when pb is not 64-aligned, else
//            its run sum.
//   interior run sums rk[k], k = A0/64 + 1 .. B1/64 - 2.
//   combine  V = xor_r v_r * x^(8*64*(n-1-r)): four interleaved Horner streams (fold x^(8*256)),
//            run groups of four read as one 16-B load aligned to the record's last run (elements
//            before run 0 count as zero), streams merged by x^(8*64), x^(8*128).
//   un-shift the register at pb is V * x^(-8(B1-pb)) (nibble sets of x^(-8*2^k), crc32_layout.h);
//            the CRC is its complement.
// Model: tests/kernel_model.py RegionModel (checked against zlib on the CPU).
#pragma once
#include <hip/hip_runtime.h>

// A/B probe builds (tools/ab_build.sh AB_FLAGS=-DAMBRY_REGION_PROBE=n; timing only, wrong CRCs):
// 1 = records not CRC'd (parse alone), 2 = no run-sum loads, 3 = no head / tail loads.
#include <stdint.h>

#include "crc32_kernels.h"
#include "crc32_layout.h"

namespace ambrycrc {
namespace region {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// LDS (besides T0..T3, one copy: t[256j + b], crc_img.h stage_slice_tables): 11 nibble sets,
// POW[4..8] (x^(8*16) .. x^(8*256)) then x^(-8*2^k), k = 0..5.
constexpr uint32_t kNibWords = kNibSetBytes / 4;  // 128
constexpr uint32_t kSets = 5 + kInvPowSets;
constexpr uint32_t kP16 = 0, kP32 = 1, kP64 = 2, kP128 = 3, kP256 = 4, kInv0 = 5;
// After the sets: x^(8*2^k), k = 0..63 (the image's power words), for the wave-wide record CRC's
// shift constants without a dependent global load each.
constexpr uint32_t kXpOff = kSets * kNibWords;
constexpr uint32_t kNibTotal = kXpOff + 64;

__device__ __forceinline__ uint32_t nmul(const uint32_t* __restrict__ nib, uint32_t v, uint32_t set) {
  const uint32_t* s = nib + set * kNibWords;
  uint32_t x = 0;
#pragma unroll
  for (int n = 0; n < 8; ++n) x ^= s[16 * n + __builtin_amdgcn_ubfe(v, 4 * n, 4)];
  return x;
}

__device__ __forceinline__ uint32_t step4(const uint32_t* __restrict__ t, uint32_t x) {
  return t[768 + (x & 0xffu)] ^ t[512 + ((x >> 8) & 0xffu)] ^ t[256 + ((x >> 16) & 0xffu)] ^ t[x >> 24];
}

// Slice-by-4 table access for hash_run / record_crc. TabC: the compact one-copy tables t[256j + b]
// (stage_slice_tables; lanes looking up different bytes conflict on LDS banks). TabR: the
// lane-column replicated slice tables of the streaming kernels (crc32_layout.h: T_j[b] at
// (j>>1)<<16 | b<<8 | (j&1)<<7 | (lane&31)<<2), conflict-free -- the one-pass kernel's processors
// use them so their lookups do not take LDS cycles from the streamers beside them.
struct TabC {
  const uint32_t* __restrict__ t;
  __device__ __forceinline__ uint32_t step4(uint32_t x) const { return region::step4(t, x); }
  __device__ __forceinline__ uint32_t t0(uint32_t b) const { return t[b]; }
};
struct TabR {
  const uint8_t* __restrict__ lds;  // the slice tables' base
  uint32_t col;                     // (lane & 31) << 2
  __device__ __forceinline__ uint32_t ld(uint32_t a) const { return *reinterpret_cast<const uint32_t*>(lds + a); }
  __device__ __forceinline__ uint32_t step4(uint32_t x) const {
    return ld((1u << 16) | (1u << 7) | ((x & 0xffu) << 8) | col) ^ ld((1u << 16) | (((x >> 8) & 0xffu) << 8) | col) ^
           ld((1u << 7) | (((x >> 16) & 0xffu) << 8) | col) ^ ld(((x >> 24) << 8) | col);
  }
  __device__ __forceinline__ uint32_t t0(uint32_t b) const { return ld((b << 8) | col); }
};

// Lane (l - 2^LVL)'s v, for lanes with bit LVL set (others: 0): DPP row shifts, then row broadcasts.
template <int LVL>
__device__ __forceinline__ uint32_t left_partner(uint32_t v) {
  if constexpr (LVL < 4) return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x110 + (1 << LVL), 0xf, 0xf, false);
  else if constexpr (LVL == 4) return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xa, 0xf, false);
  else return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xc, 0xf, false);
}

// Bytes of a little-endian word w at run byte offsets [4w, 4w + 4) with offset >= lo / < hi.
__device__ __forceinline__ uint32_t keep_ge(int d) {  // bytes at index >= d (d = lo - 4w)
  return d <= 0 ? 0xFFFFFFFFu : (d >= 4 ? 0u : (0xFFFFFFFFu << (8 * d)));
}
__device__ __forceinline__ uint32_t keep_lt(int d) {  // bytes at index < d (d = hi - 4w)
  return d >= 4 ? 0xFFFFFFFFu : (d <= 0 ? 0u : (0xFFFFFFFFu >> (32 - 8 * d)));
}

// The 16-B pieces of the 64-B run at base + r0 that hold bytes of [lo, hi) (others zero).
__device__ __forceinline__ void load_run(const uint8_t* __restrict__ base, uint64_t r0, int lo, int hi, u32x4 (&w)[4]) {
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    w[q] = u32x4{0u, 0u, 0u, 0u};
#if AMBRY_REGION_PROBE != 3  // probe 3 (timing only, wrong CRCs): no head / tail loads
    if (16 * q + 16 > lo && 16 * q < hi) w[q] = *reinterpret_cast<const u32x4*>(base + r0 + 16 * q);
#endif
  }
}

// Raw CRC register at the end of that run over its bytes [lo, hi) (others zero), with 0xFF XORed
// into bytes [lo, lo + ninit): four independent 4-step chains, one per piece, merged by x^(8*16)
// and x^(8*32) (depth 4 + 2 instead of 16 dependent steps).
template <class Tab>
__device__ __forceinline__ uint32_t hash_run(const Tab& t, const uint32_t* __restrict__ nib, const u32x4 (&w)[4],
                                             int lo, int hi, int ninit) {
  uint32_t p[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    uint32_t s = 0;
#pragma unroll
    for (int d = 0; d < 4; ++d) {
      const int o = 16 * q + 4 * d;
      uint32_t v = w[q][d] & keep_ge(lo - o) & keep_lt(hi - o);
      v ^= keep_ge(lo - o) & keep_lt(lo + ninit - o);
      s = t.step4(s ^ v);
    }
    p[q] = s;
  }
  return nmul(nib, nmul(nib, p[0], kP16) ^ p[1], kP32) ^ nmul(nib, p[2], kP16) ^ p[3];
}

// Stage the nibble sets into nib[kSets * kNibWords] (the caller syncs).
__device__ __forceinline__ void stage_nib(uint32_t* __restrict__ nib, const uint32_t* __restrict__ img) {
  if (threadIdx.x < 64) nib[kXpOff + threadIdx.x] = img[kLdsBytes / 4 + threadIdx.x];
  for (uint32_t i = threadIdx.x; i < kSets * kNibWords; i += blockDim.x) {
    const uint32_t set = i / kNibWords, w = i % kNibWords;
    const uint32_t byte = set < 5 ? kNibBase + kPowOff + kNibSetBytes * (4 + set) : kImgInvOff + kNibSetBytes * (set - 5);
    nib[i] = img[byte / 4 + w];
  }
}

// Pass 2's extra LDS words (crc32_layout.h kImgRegOff; region_msg_kernel stages them): hm = H0,
// GE, LT (kRegAuxWords), bt = the byte tables of x^(8*256). NoAux: nibble forms only (the
// one-pass processors, whose LDS holds the streamers' replicated tables).
struct NoAux {
  static constexpr bool kOn = false, kMask = false, kByte = false, kUn = false;
  const uint32_t* hm = nullptr;
  const uint32_t* bt = nullptr;
  const uint32_t* un = nullptr;
};
struct Aux {
  static constexpr bool kOn = true, kMask = (AMBRY_REGION_AUX & 1) != 0, kByte = (AMBRY_REGION_AUX & 2) != 0,
                        kUn = (AMBRY_REGION_AUX & 4) != 0;
  const uint32_t* __restrict__ hm;
  const uint32_t* __restrict__ bt;
  const uint32_t* __restrict__ un;  // un-shift sets: x^(-8 d0) (0..7), x^(-64 d1) (8..15)
};

// The image's kRegWords region words into hm, bt and un (the caller syncs).
__device__ __forceinline__ void stage_aux(uint32_t* __restrict__ hm, uint32_t* __restrict__ bt,
                                          uint32_t* __restrict__ un, const uint32_t* __restrict__ img) {
  const uint32_t* src = img + kImgRegOff / 4;
  for (uint32_t i = threadIdx.x; i < kRegWords; i += blockDim.x) {
    if (i < kRegAuxWords)
      hm[i] = src[i];
    else if (i < kRegAuxWords + kRegByteWords)
      bt[i - kRegAuxWords] = src[i];
    else
      un[i - kRegAuxWords - kRegByteWords] = src[i];
  }
}

// v * x^(8*256) from the byte tables: four lookups (byte-indexed, one VALU address each) where
// the nibble sets take eight.
__device__ __forceinline__ uint32_t bmul(const uint32_t* __restrict__ bt, uint32_t v) {
  return bt[v & 0xffu] ^ bt[256 + ((v >> 8) & 0xffu)] ^ bt[512 + ((v >> 16) & 0xffu)] ^ bt[768 + (v >> 24)];
}

// hash_run with each word's byte mask read from LDS -- LT / GE at the byte offset clamped into
// the word, one v_med3 and one broadcast read per mask -- in place of the compares and shifts of
// keep_ge / keep_lt (about half of a record's VALU work in pass 2), and without the initial-register
// bytes: the caller XORs H0[lo] (the raw register is linear in the bytes). LO0: bytes from 0 (tail
// runs, no GE mask).
template <bool LO0, class Tab>
__device__ __forceinline__ uint32_t hash_run_m(const Tab& t, const uint32_t* __restrict__ nib,
                                               const uint32_t* __restrict__ hm, const u32x4 (&w)[4], int lo, int hi) {
  const int lo4 = 4 * lo, hi4 = 4 * hi;
  uint32_t p[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    uint32_t s = 0;
#pragma unroll
    for (int d = 0; d < 4; ++d) {
      const int c = 16 * (4 * q + d);  // 4 x the word's first byte offset
      uint32_t v = w[q][d] & hm[kRegLt + ((min(max(hi4, c), c + 16) - c) >> 2)];
      if (!LO0) v &= hm[kRegGe + ((min(max(lo4, c), c + 16) - c) >> 2)];
      s = t.step4(s ^ v);
    }
    p[q] = s;
  }
  return nmul(nib, nmul(nib, p[0], kP16) ^ p[1], kP32) ^ nmul(nib, p[2], kP16) ^ p[3];
}

// Four run groups (16 run sums) from group g on, as 16-B loads; groups past ng are not read.
__device__ __forceinline__ void load_groups(const uint32_t* __restrict__ rk, int64_t e0, int64_t g, int64_t ng,
                                            u32x4 (&r)[4]) {
#pragma unroll
  for (int u = 0; u < 4; ++u) {
#if AMBRY_REGION_PROBE == 2  // probe 2 (timing only, wrong CRCs): no run-sum loads
    r[u] = u32x4{(uint32_t)g, 0u, 0u, (uint32_t)u};
#else
    if (g + u < ng) __builtin_memcpy(&r[u], rk + e0 + 4 * (g + u), 16);
#endif
  }
}

// zlib CRC-32 of the len bytes at offset pa from base; rk = RegionArgs::rk + kRunPad. Every load
// is issued before the first is used (head and tail runs, the first 16 run sums), and each
// Horner step group prefetches the next 16 sums.
// X = Aux: head / tail runs by hash_run_m plus H0[lo], Horner steps by the byte tables.
template <class Tab, class X = NoAux>
__device__ __forceinline__ uint32_t record_crc(const Tab& t, const uint32_t* __restrict__ nib,
                                               const uint8_t* __restrict__ base, const uint32_t* __restrict__ rk,
                                               uint64_t pa, uint64_t len, const X& x = X{}) {
  if (len == 0) return 0;
  const uint64_t pb = pa + len;
  if (len < 4) {
    uint32_t c = 0xFFFFFFFFu;
    for (uint64_t i = pa; i < pb; ++i) c = t.t0((c ^ base[i]) & 0xffu) ^ (c >> 8);
    return ~c;
  }
  const uint64_t A0 = pa & ~uint64_t(63), B1 = (pb + 63) & ~uint64_t(63);
  const int64_t n = (int64_t)((B1 - A0) >> 6), k0 = (int64_t)(A0 >> 6);
  const int lo = (int)(pa - A0), hi = pb - A0 < 64 ? (int)(pb - A0) : 64;
  const int tin = hi - lo;
  const bool tail_bytes = n >= 2 && (pb & 63u) != 0;
  const int thi = (int)(pb - (B1 - 64));
  const int64_t ng = (n + 3) >> 2, e0 = k0 + n - 4 * ng;
  u32x4 hw[4], tw[4], nxt[4];
  load_run(base, A0, lo, hi, hw);
  load_run(base, B1 - 64, 0, tail_bytes ? thi : 0, tw);
  load_groups(rk, e0, 0, ng, nxt);
  uint32_t H, T;
  if constexpr (X::kMask) {
    H = hash_run_m<false>(t, nib, x.hm, hw, lo, hi) ^ x.hm[kRegH0 + lo];
    T = tail_bytes ? hash_run_m<true>(t, nib, x.hm, tw, 0, thi) : 0u;
  } else {
    H = hash_run(t, nib, hw, lo, hi, tin < 4 ? tin : 4);
    T = tail_bytes ? hash_run(t, nib, tw, 0, thi, 0) : 0u;
  }
  if (tin < 4) H ^= 0xFFFFFFFFu >> (8 * tin);
  // Horner over runs k0 .. k0+n-1 in groups of four ending at the last run. The head run and the
  // first group's padding (runs before k0, zero) are patched into group 0's sums once; the tail
  // run enters with factor 1 (it is the last), so the raw sum the loop folds in is swapped for T
  // after it. The loop itself is four lookups and four XORs per run.
  const int32_t n32 = (int32_t)n, ng32 = (int32_t)ng, rb = n32 - 4 * ng32;  // rb: -3..0
  const uint32_t rlast = tail_bytes ? rk[k0 + n - 1] : 0u;
#pragma unroll
  for (int q = 0; q < 4; ++q) nxt[0][q] = rb + q < 0 ? 0u : rb + q == 0 ? H : nxt[0][q];
  uint32_t s0 = 0, s1 = 0, s2 = 0, s3 = 0;  // s3: the stream updated last
  for (int32_t g = 0; g < ng32; g += 4) {
    u32x4 r[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) r[u] = nxt[u];
    if (g + 4 < ng32) load_groups(rk, e0, g + 4, ng, nxt);
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      if (g + u < ng32) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          uint32_t nv;
          if constexpr (X::kByte)
            nv = bmul(x.bt, s0) ^ r[u][q];
          else
            nv = nmul(nib, s0, kP256) ^ r[u][q];
          s0 = s1;
          s1 = s2;
          s2 = s3;
          s3 = nv;
        }
      }
    }
  }
  s3 ^= T ^ rlast;
  // streams merged by x^(8*64) (s0 * x^(8*192) ^ s1 * x^(8*128) ^ s2 * x^(8*64) ^ s3), then the
  // register at B1 un-shifted to pb
  uint32_t V = s3 ^ nmul(nib, s2 ^ nmul(nib, s1 ^ nmul(nib, s0, kP64), kP64), kP64);
  const uint32_t d = (uint32_t)(B1 - pb);
  if constexpr (X::kUn) {
    V = nmul(x.un, nmul(x.un, V, d & 7u), 8u + (d >> 3));
  } else {
#pragma unroll
    for (uint32_t k = 0; k < kInvPowSets; ++k)
      if (d & (1u << k)) V = nmul(nib, V, kInv0 + k);
  }
  return ~V;
}

// record_crc in two steps, for the one-pass processors (AMBRY_FUSED_ENDS): record_ends hashes the
// head and tail runs from the bytes -- right after the parse, whose loads fetched those lines, and
// before the wait for the run sums, which the streamers' nontemporal loads outlast in L2 -- and
// record_crc_from_ends does the rest once the sums exist. Records under 4 bytes: the CRC itself
// in h.
struct RecEnds {
  uint32_t h, t;
};
template <class Tab>
__device__ __forceinline__ RecEnds record_ends(const Tab& t, const uint32_t* __restrict__ nib,
                                               const uint8_t* __restrict__ base, uint64_t pa, uint64_t len) {
  if (len == 0) return RecEnds{0u, 0u};
  const uint64_t pb = pa + len;
  if (len < 4) {
    uint32_t c = 0xFFFFFFFFu;
    for (uint64_t i = pa; i < pb; ++i) c = t.t0((c ^ base[i]) & 0xffu) ^ (c >> 8);
    return RecEnds{~c, 0u};
  }
  const uint64_t A0 = pa & ~uint64_t(63), B1 = (pb + 63) & ~uint64_t(63);
  const int64_t n = (int64_t)((B1 - A0) >> 6);
  const int lo = (int)(pa - A0), hi = pb - A0 < 64 ? (int)(pb - A0) : 64;
  const int tin = hi - lo;
  const bool tail_bytes = n >= 2 && (pb & 63u) != 0;
  const int thi = (int)(pb - (B1 - 64));
  u32x4 hw[4], tw[4];
  load_run(base, A0, lo, hi, hw);
  load_run(base, B1 - 64, 0, tail_bytes ? thi : 0, tw);
  uint32_t H = hash_run(t, nib, hw, lo, hi, tin < 4 ? tin : 4);
  if (tin < 4) H ^= 0xFFFFFFFFu >> (8 * tin);
  return RecEnds{H, tail_bytes ? hash_run(t, nib, tw, 0, thi, 0) : 0u};
}

__device__ __forceinline__ uint32_t record_crc_from_ends(const uint32_t* __restrict__ nib,
                                                         const uint32_t* __restrict__ rk, uint64_t pa, uint64_t len,
                                                         RecEnds e) {
  if (len < 4) return e.h;
  const uint64_t pb = pa + len;
  const uint64_t A0 = pa & ~uint64_t(63), B1 = (pb + 63) & ~uint64_t(63);
  const int64_t n = (int64_t)((B1 - A0) >> 6), k0 = (int64_t)(A0 >> 6);
  const bool tail_bytes = n >= 2 && (pb & 63u) != 0;
  const int64_t ng = (n + 3) >> 2, e0 = k0 + n - 4 * ng;
  u32x4 nxt[4];
  load_groups(rk, e0, 0, ng, nxt);
  const int32_t n32 = (int32_t)n, ng32 = (int32_t)ng, rb = n32 - 4 * ng32;
  const uint32_t rlast = tail_bytes ? rk[k0 + n - 1] : 0u;
#pragma unroll
  for (int q = 0; q < 4; ++q) nxt[0][q] = rb + q < 0 ? 0u : rb + q == 0 ? e.h : nxt[0][q];
  uint32_t s0 = 0, s1 = 0, s2 = 0, s3 = 0;
  for (int32_t g = 0; g < ng32; g += 4) {
    u32x4 r[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) r[u] = nxt[u];
    if (g + 4 < ng32) load_groups(rk, e0, g + 4, ng, nxt);
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      if (g + u < ng32) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const uint32_t nv = nmul(nib, s0, kP256) ^ r[u][q];
          s0 = s1;
          s1 = s2;
          s2 = s3;
          s3 = nv;
        }
      }
    }
  }
  s3 ^= e.t ^ rlast;
  uint32_t V = s3 ^ nmul(nib, s2 ^ nmul(nib, s1 ^ nmul(nib, s0, kP64), kP64), kP64);
  const uint32_t d = (uint32_t)(B1 - pb);
#pragma unroll
  for (uint32_t k = 0; k < kInvPowSets; ++k)
    if (d & (1u << k)) V = nmul(nib, V, kInv0 + k);
  return ~V;
}

// LDS sets: x^(8*64*2^k) for k = 0..5 (the tree), x^(8*4096) (the fold): the image's POW[6..12].
// x^(8*2^(6+s)) for s = 0..10 (the image's POW[6..16]): record_crc_direct's tree (s = 0..5,
// 64-B runs) and fold (s = 6); record_crc_runs_wave's in-lane fold of 64-B runs (s = 0), tree of
// 256-B lane slices (s = 2..7), round combine (s = 8) and stream fold (s = 10).
constexpr uint32_t kDirSets = 11;
constexpr uint32_t kDirRun = 0, kDirRunTree = 2, kDirRound = 8, kDirStream = 10;
// Records of more runs than this go to the whole wave (record_crc_runs_wave).
constexpr int64_t kLongRuns = 512;
constexpr uint32_t kDirFold = 6;
__device__ __forceinline__ void stage_direct_nib(uint32_t* __restrict__ dn, const uint32_t* __restrict__ img) {
  for (uint32_t i = threadIdx.x; i < kDirSets * kNibWords; i += blockDim.x) {
    const uint32_t set = i / kNibWords, w = i % kNibWords;
    dn[i] = img[(kNibBase + kPowOff + kNibSetBytes * (6 + set)) / 4 + w];
  }
}

// zlib CRC-32 of a long record by the whole wave from the run sums (every lane the same pa, len;
// len >= 4): the record's runs [A0, B1) as record_crc takes them (head and tail runs from the
// bytes, the interior from rk), in rounds of 256 aligned to the record's last run -- lane l takes
// runs 4l .. 4l + 3 of a round (one 16-B load of sums, folded by x^(8*64)) -- four streams of rounds
// folded by x^(8*65536), combined by x^(8*16384), the lanes merged by the tree over 256-B slices
// (x^(8*256*2^k)) from dn's LDS sets (lane 63 ends at B1), then un-shifted to the record's end.
// Nibble multiplies only: round 3's form (per-lane slices of variable length) needed gf2_mul
// shifts -- 32-round loops -- for its tree.
template <class Tab>
__device__ __forceinline__ uint32_t record_crc_runs_wave(const Tab& t, const uint32_t* __restrict__ nib,
                                                         const uint32_t* __restrict__ dn,
                                                         const uint8_t* __restrict__ base,
                                                         const uint32_t* __restrict__ rk, uint64_t pa, uint64_t len,
                                                         uint32_t lane) {
  const uint64_t pb = pa + len;
  const uint64_t A0 = pa & ~uint64_t(63), B1 = (pb + 63) & ~uint64_t(63);
  const int64_t n = (int64_t)((B1 - A0) >> 6), k0 = (int64_t)(A0 >> 6);
  const int lo = (int)(pa - A0), hi = pb - A0 < 64 ? (int)(pb - A0) : 64;
  const int tin = hi - lo;
  const bool tail_bytes = n >= 2 && (pb & 63u) != 0;
  const int thi = (int)(pb - (B1 - 64));
  u32x4 hw[4], tw[4];
  load_run(base, A0, lo, hi, hw);
  load_run(base, B1 - 64, 0, tail_bytes ? thi : 0, tw);
  uint32_t H = hash_run(t, nib, hw, lo, hi, tin < 4 ? tin : 4);
  if (tin < 4) H ^= 0xFFFFFFFFu >> (8 * tin);
  const uint32_t T = tail_bytes ? hash_run(t, nib, tw, 0, thi, 0) : 0u;
  // Rounds of 256 runs, lane l taking runs 4l .. 4l + 3 of each (one 16-B load of sums, folded in
  // the lane by x^(8*64)), V rounds padded at the front to a multiple of four; round v feeds stream
  // v mod 4, each folded by x^(8*65536): four independent chains, eight rounds' sums in flight.
  // (A run a lane a round took one 4-B load each: ~64 round trips per 4 MiB record.)
  const int64_t V = (((n + 255) >> 8) + 3) & ~int64_t(3);
  uint32_t s0 = 0, s1 = 0, s2 = 0, s3 = 0;
  for (int64_t v0 = 0; v0 < V; v0 += 8) {
    u32x4 sum[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int64_t r0 = n - 256 * (V - (v0 + u)) + 4 * (int64_t)lane;
      sum[u] = u32x4{0u, 0u, 0u, 0u};
      if (v0 + u < V && r0 + 3 >= 1) __builtin_memcpy(&sum[u], rk + k0 + r0, 16);  // r0 >= -3: inside rk's pad
    }
#pragma unroll
    for (int u = 0; u < 8; u += 4) {
      if (v0 + u >= V) break;
      uint32_t w[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int64_t r0 = n - 256 * (V - (v0 + u + q)) + 4 * (int64_t)lane;
        uint32_t x = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int64_t r = r0 + j;
          const uint32_t val = r < 0 ? 0u : r == 0 ? H : (r == n - 1 && tail_bytes) ? T : sum[u + q][j];
          x = j ? nmul(dn, x, kDirRun) ^ val : val;
        }
        w[q] = x;
      }
      s0 = nmul(dn, s0, kDirStream) ^ w[0];
      s1 = nmul(dn, s1, kDirStream) ^ w[1];
      s2 = nmul(dn, s2, kDirStream) ^ w[2];
      s3 = nmul(dn, s3, kDirStream) ^ w[3];
    }
  }
  uint32_t acc = nmul(dn, nmul(dn, nmul(dn, s0, kDirRound) ^ s1, kDirRound) ^ s2, kDirRound) ^ s3;
  {
    const uint32_t pt = left_partner<0>(acc);
    if (lane & 1u) acc ^= nmul(dn, pt, kDirRunTree + 0);
  }
  {
    const uint32_t pt = left_partner<1>(acc);
    if (lane & 2u) acc ^= nmul(dn, pt, kDirRunTree + 1);
  }
  {
    const uint32_t pt = left_partner<2>(acc);
    if (lane & 4u) acc ^= nmul(dn, pt, kDirRunTree + 2);
  }
  {
    const uint32_t pt = left_partner<3>(acc);
    if (lane & 8u) acc ^= nmul(dn, pt, kDirRunTree + 3);
  }
  {
    const uint32_t pt = left_partner<4>(acc);
    if (lane & 16u) acc ^= nmul(dn, pt, kDirRunTree + 4);
  }
  {
    const uint32_t pt = left_partner<5>(acc);
    if (lane & 32u) acc ^= nmul(dn, pt, kDirRunTree + 5);
  }
  uint32_t Vv = __builtin_amdgcn_readlane(acc, 63);
  const uint32_t d = (uint32_t)(B1 - pb);
#pragma unroll
  for (uint32_t k = 0; k < kInvPowSets; ++k)
    if (d & (1u << k)) Vv = nmul(nib, Vv, kInv0 + k);
  return ~Vv;
}

__device__ __forceinline__ uint32_t record_crc(const uint32_t* __restrict__ t, const uint32_t* __restrict__ nib,
                                               const uint8_t* __restrict__ base, const uint32_t* __restrict__ rk,
                                               uint64_t pa, uint64_t len) {
  return record_crc(TabC{t}, nib, base, rk, pa, len);
}

// Appends a long record to the grid-wide list (region_long_kernel, message_kernels.hip) for one
// thread's message (region_msg_kernel: a thread per message, its own atomic result, no broadcast);
// false when the list is full (the caller then takes the record itself).
__device__ __forceinline__ bool list_long(const LongList& l, uint64_t pa, uint64_t len, uint32_t ex, uint64_t msg,
                                          uint32_t bit) {
  const uint32_t pieces = (uint32_t)((len + kLongPiece - 1) / kLongPiece);
  if (pieces > kLongMaxPieces) return false;
  const unsigned long long was = atomicAdd(l.ctr, (1ull << 32) | pieces);
  const uint32_t at = (uint32_t)(was >> 32);
  if (at >= l.cap) return false;
  const bool room = (uint64_t)(uint32_t)was + pieces <= l.pcap;
  LongRec& lr = l.rec[at];
  lr.pa = pa;
  lr.msg = msg;
  lr.len = (uint32_t)len;
  lr.ex = ex;
  lr.bit = bit;
  lr.piece0 = (uint32_t)was;
  lr.pieces = room ? pieces : 0;  // no slots left: listed empty, taken by the caller
  lr.done = 0;
  return room;
}

// The same for a whole wave with wave-uniform arguments (the region processors): every lane runs the
// atomic (lane 0 adds, the rest add 0) and lane 0's result is broadcast, so the return value is
// wave-uniform without a lane-0-only branch before a readfirstlane. Lane 0 writes
// the record.
__device__ __forceinline__ bool list_long_wave(const LongList& l, uint64_t pa, uint64_t len, uint32_t ex,
                                               uint64_t msg, uint32_t bit, uint32_t lane) {
  const uint32_t pieces = (uint32_t)((len + kLongPiece - 1) / kLongPiece);
  if (pieces > kLongMaxPieces) return false;
  const unsigned long long inc = lane == 0 ? ((1ull << 32) | pieces) : 0ull;
  const unsigned long long raw = atomicAdd(l.ctr, inc);
  const unsigned long long was = ((unsigned long long)__builtin_amdgcn_readfirstlane((uint32_t)(raw >> 32)) << 32) |
                                 __builtin_amdgcn_readfirstlane((uint32_t)raw);
  const uint32_t at = (uint32_t)(was >> 32);
  if (at >= l.cap) return false;
  const bool room = (uint64_t)(uint32_t)was + pieces <= l.pcap;
  if (lane == 0) {
    LongRec& lr = l.rec[at];
    lr.pa = pa;
    lr.msg = msg;
    lr.len = (uint32_t)len;
    lr.ex = ex;
    lr.bit = bit;
    lr.piece0 = (uint32_t)was;
    lr.pieces = room ? pieces : 0;  // no slots left: listed empty, taken by the caller
    lr.done = 0;
  }
  return room;
}

}  // namespace region
}  // namespace ambrycrc
