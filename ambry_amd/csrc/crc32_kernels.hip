// crc32_kernels.hip -- gfx950 (CDNA4) kernels for Ambry's blob CRC-32 path.
//
// Replaces, for device-resident batches of chunks, the byte loop of
// ambry-utils/.../utils/Crc32.java:55-143 (and java.util.zip.CRC32.update, the
// same function) as called per router chunk (ambry-router/.../PutOperation.java:
// 1700-1703, 2033-2054) and per blob record (ambry-messageformat/.../
// MessageFormatRecord.java:1797-1832). Results are bit-exact CRC-32/ISO-HDLC.
//
// Work decomposition
//   chunk  -> tiles of <= 2^tile_log2 bytes, aligned to the chunk's 16-B-aligned
//             end (so every tile but the first is a whole number of 16-B pieces)
//   tile   -> one wavefront; the wave sweeps the tile in 1 KiB blocks, lane l
//             owning bytes [16l, 16l+16) of every block (one coalesced
//             global_load_dwordx4 per block per lane)
//   lane   -> slice-by-4 over its 16-B piece using LDS byte tables that one
//             v_perm_b32 addresses; the lane state hops one block with an
//             x^(8*1024) nibble-table multiply (independent of the piece's own
//             table walk, so consecutive pieces overlap)
//   wave   -> 6-level xor-shuffle tree, level l shifting by 16*2^l bytes
//   tile   -> shifted by its distance to the chunk end and atomically XORed into
//             out[chunk] (XOR is exact and order-free => deterministic)
//
// LDS layout: crc32_layout.h. One 1024-thread workgroup per CU (the image is
// ~150 KiB), persistent over the tile list.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "crc32_gf2.h"
#include "crc32_layout.h"
#include "crc32_kernels.h"

namespace ambrycrc {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__shared__ __attribute__((aligned(16))) uint32_t g_lds[kLdsBytes / 4];

__device__ __forceinline__ uint32_t lds_rd(uint32_t byte_addr) {
  return *reinterpret_cast<const uint32_t*>(reinterpret_cast<const char*>(g_lds) + byte_addr);
}

__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}

// Per-lane address constants for slice table j: region bit, (j&1)*128, lane column.
struct LaneConst {
  uint32_t L0, L1, L2, L3;
};

__device__ __forceinline__ LaneConst make_lane_const(uint32_t lane) {
  const uint32_t col = (lane & 31u) << 2;
  LaneConst k;
  k.L0 = (0u << 16) | (0u << 7) | col;
  k.L1 = (0u << 16) | (1u << 7) | col;
  k.L2 = (1u << 16) | (0u << 7) | col;
  k.L3 = (1u << 16) | (1u << 7) | col;
  return k;
}

// One slice-by-4 step on x = state ^ word: T3[x.b0]^T2[x.b1]^T1[x.b2]^T0[x.b3] ^ xin.
// perm(L, x, sel): result byte0 = L.b0 (lane column), byte1 = x.b_k, byte2 = L.b2 (region), byte3 = 0.
__device__ __forceinline__ uint32_t slice4(uint32_t x, const LaneConst& k, uint32_t xin) {
  const uint32_t a0 = __builtin_amdgcn_perm(k.L3, x, 0x0C060004u);
  const uint32_t a1 = __builtin_amdgcn_perm(k.L2, x, 0x0C060104u);
  const uint32_t a2 = __builtin_amdgcn_perm(k.L1, x, 0x0C060204u);
  const uint32_t a3 = __builtin_amdgcn_perm(k.L0, x, 0x0C060304u);
  const uint32_t t = xor3(lds_rd(a0), lds_rd(a1), lds_rd(a2));
  return xor3(t, lds_rd(a3), xin);
}

// Raw CRC (zero register, no xor-out) of one 16-B piece, xor xin.
__device__ __forceinline__ uint32_t rpiece(u32x4 w, const LaneConst& k, uint32_t xin) {
  uint32_t s = slice4(w.x, k, w.y);
  s = slice4(s, k, w.z);
  s = slice4(s, k, w.w);
  return slice4(s, k, xin);
}

// v * C mod P where C's nibble tables sit at kNibBase + set_off (conflict-free, 8 lookups).
__device__ __forceinline__ uint32_t nib_mul(uint32_t v, uint32_t set_off) {
  uint32_t t[8];
#pragma unroll
  for (int n = 0; n < 8; ++n)
    t[n] = lds_rd(kNibBase + set_off + 64u * n + (__builtin_amdgcn_ubfe(v, 4 * n, 4) << 2));
  return xor3(xor3(t[0], t[1], t[2]), xor3(t[3], t[4], t[5]), t[6] ^ t[7]);
}

// v * x^(8n) mod P for a wave-uniform n (register advanced over n zero bytes).
__device__ __forceinline__ uint32_t shift_bytes(uint32_t v, uint64_t n, const uint32_t* __restrict__ xpow2) {
  while (n) {
    const uint32_t k = (uint32_t)__builtin_ctzll(n);
    n &= n - 1;
    v = (k < kPowTables) ? nib_mul(v, kPowOff + kNibSetBytes * k) : gf2_mul(v, xpow2[k]);
  }
  return v;
}

template <bool NT>
__device__ __forceinline__ u32x4 ld16(const u32x4* p) {
  if constexpr (NT) {
    return __builtin_nontemporal_load(p);
  } else {
    return *p;
  }
}

// Raw CRC of body [bs, be) (be 16-aligned, bs <= be arbitrary), returned in lane 63
// (other lanes: junk). Bytes below bs are treated as zeros, which leave a zero
// register unchanged, so the virtual range is aligned down to whole 1 KiB blocks.
template <int U, bool NT>
__device__ __forceinline__ uint32_t body_crc(const uint8_t* __restrict__ base, uint64_t bs, uint64_t be,
                                             uint32_t lane, const LaneConst& k) {
  const uint64_t nb = (be - bs + kBlockBytes - 1) / kBlockBytes;
  if (nb == 0) return 0u;
  // The virtual start may precede the allocation (chunk in its first KiB): signed
  // arithmetic, and only lanes whose piece reaches bs ever form a load address.
  const int64_t v0 = (int64_t)be - (int64_t)(nb * kBlockBytes);
  const u32x4* q = reinterpret_cast<const u32x4*>(base + v0) + lane;

  // Block 0 carries the (possibly unaligned) start: mask what lies before bs.
  u32x4 w = {0u, 0u, 0u, 0u};
  const int64_t p = v0 + 16 * (int64_t)lane;
  if (p + 16 > (int64_t)bs) {  // => p >= floor16(bs) >= 0: inside the caller's buffer
    w = ld16<NT>(reinterpret_cast<const u32x4*>(base + p));
    if (p < (int64_t)bs) {
      const uint32_t cut = (uint32_t)(bs - p);  // 1..15 leading bytes to drop
#pragma unroll
      for (int d = 0; d < 4; ++d) {
        const int lo = (int)cut - 4 * d;  // bytes of dword d to drop
        const uint32_t m = lo <= 0 ? 0xFFFFFFFFu : (lo >= 4 ? 0u : (0xFFFFFFFFu << (8 * lo)));
        w[d] &= m;
      }
    }
  }
  uint32_t s = rpiece(w, k, 0u);

  uint64_t b = 1;
  for (; b + U <= nb; b += U) {
    u32x4 buf[U];
#pragma unroll
    for (int u = 0; u < U; ++u) buf[u] = ld16<NT>(q + (b + u) * (kBlockBytes / 16));
#pragma unroll
    for (int u = 0; u < U; ++u) s = rpiece(buf[u], k, nib_mul(s, kFoldOff));
  }
  for (; b < nb; ++b) {
    const u32x4 x = ld16<NT>(q + b * (kBlockBytes / 16));
    s = rpiece(x, k, nib_mul(s, kFoldOff));
  }

  // Lane l's stream ends 16(63-l) bytes before be: xor-tree with shifts 16*2^lvl.
#pragma unroll
  for (int lvl = 0; lvl < 6; ++lvl) {
    const uint32_t o = __shfl_xor(s, 1 << lvl);
    const uint32_t sh = nib_mul(o, kTreeOff + kNibSetBytes * lvl);
    s = (lane & (1u << lvl)) ? (s ^ sh) : s;
  }
  return s;
}

// Find chunk c with tile_start[c] <= t < tile_start[c+1], searching [lo, n).
__device__ __forceinline__ uint32_t find_chunk(const uint32_t* __restrict__ tile_start, uint32_t n, uint32_t t,
                                               uint32_t lo, uint32_t lane) {
  uint32_t hi = n;
  while (hi - lo > 1) {
    const uint32_t step = (hi - lo + 63) / 64;
    const uint32_t idx = lo + lane * step;
    const bool ok = idx < hi && tile_start[idx] <= t;
    const uint64_t m = __ballot(ok);
    const uint32_t last = 63u - (uint32_t)__builtin_clzll(m);
    const uint32_t nlo = lo + last * step;
    const uint32_t nhi = lo + (last + 1) * step;
    lo = nlo;
    hi = nhi < hi ? nhi : hi;
  }
  return lo;
}

__device__ __forceinline__ uint64_t aligned_end(uint64_t s, uint64_t e) {
  uint64_t b = e & ~uint64_t(15);
  return b < s ? s : b;
}

template <int U, bool NT>
__global__ __launch_bounds__(1024) void crc32_tiles_kernel(TilesArgs a) {
  // Stage the table image (SLICE + nibble constants) into LDS once per workgroup.
  {
    const u32x4* src = reinterpret_cast<const u32x4*>(a.img);
    u32x4* dst = reinterpret_cast<u32x4*>(g_lds);
    for (uint32_t i = threadIdx.x; i < kLdsBytes / 16; i += blockDim.x) dst[i] = src[i];
  }
  __syncthreads();

  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t waves_per_block = blockDim.x >> 6;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(blockIdx.x * waves_per_block + (threadIdx.x >> 6));
  const uint32_t nwaves = gridDim.x * waves_per_block;
  const uint32_t total = a.tile_start[a.n];
  const uint32_t* xpow2 = a.img + kLdsBytes / 4;
  const LaneConst k = make_lane_const(lane);
  const uint64_t tile = 1ull << a.tile_log2;

  uint32_t c_lo = 0;
  for (uint32_t t = wave; t < total; t += nwaves) {
    const uint32_t c = __builtin_amdgcn_readfirstlane(find_chunk(a.tile_start, a.n, t, c_lo, lane));
    c_lo = c;
    const uint64_t cs = a.off[c];
    const uint64_t ce = cs + a.len[c];
    const uint64_t cb = aligned_end(cs, ce);
    const uint32_t nt = a.tile_start[c + 1] - a.tile_start[c];
    const uint32_t q = t - a.tile_start[c];  // 0 = first tile of the chunk
    const uint64_t m = nt - 1 - q;           // tiles after this one
    const uint64_t be = cb - m * tile;
    const uint64_t bs0 = be > tile ? be - tile : 0;
    const uint64_t bs = bs0 > cs ? bs0 : cs;

    uint32_t r = body_crc<U, NT>(a.base, bs, be, lane, k);
    r = __builtin_amdgcn_readlane(r, 63);
    r = shift_bytes(r, (ce - cb) + m * tile, xpow2);
    if (m == 0) {  // trailing <16 bytes of the chunk, byte-wise through T0 (lane column 0)
      uint32_t tr = 0;
      for (uint64_t p = cb; p < ce; ++p) tr = (tr >> 8) ^ lds_rd(((tr ^ a.base[p]) & 0xffu) << 8);
      r ^= tr;
    }
    if (q == 0) {  // initial register: ~crc_in advanced over the whole chunk, plus xor-out
      const uint32_t cin = a.crc_in ? a.crc_in[c] : 0u;
      r ^= shift_bytes(~cin, ce - cs, xpow2) ^ 0xFFFFFFFFu;
    }
    if (lane == 0) atomicXor(&a.out[c], r);
  }
}

// Exclusive scan of per-chunk tile counts (one workgroup) + zero the outputs.
__global__ __launch_bounds__(1024) void crc32_plan_kernel(PlanArgs a) {
  __shared__ uint32_t part[1024];
  const uint32_t tid = threadIdx.x;
  const uint32_t per = (a.n + 1023u) / 1024u;
  const uint32_t lo = tid * per;
  const uint32_t hi = lo + per < a.n ? lo + per : a.n;
  uint32_t sum = 0;
  for (uint32_t c = lo; c < hi; ++c) {
    const uint64_t cs = a.off[c];
    const uint64_t cb = aligned_end(cs, cs + a.len[c]);
    const uint64_t body = cb - cs;
    const uint64_t nt = (body + (1ull << a.tile_log2) - 1) >> a.tile_log2;
    sum += nt ? (uint32_t)nt : 1u;
    a.out[c] = 0u;
  }
  part[tid] = sum;
  __syncthreads();
  for (uint32_t d = 1; d < 1024; d <<= 1) {  // Hillis-Steele inclusive scan
    const uint32_t v = tid >= d ? part[tid - d] : 0u;
    __syncthreads();
    part[tid] += v;
    __syncthreads();
  }
  uint32_t run = part[tid] - sum;  // exclusive prefix of this thread's range
  for (uint32_t c = lo; c < hi; ++c) {
    a.tile_start[c] = run;
    const uint64_t cs = a.off[c];
    const uint64_t cb = aligned_end(cs, cs + a.len[c]);
    const uint64_t nt = (cb - cs + (1ull << a.tile_log2) - 1) >> a.tile_log2;
    run += nt ? (uint32_t)nt : 1u;
  }
  if (tid == 1023) a.tile_start[a.n] = part[1023];
}

__global__ void crc32_verify_kernel(const uint32_t* __restrict__ crc, const uint32_t* __restrict__ expected,
                                    uint8_t* __restrict__ mismatch, uint32_t* __restrict__ count, uint32_t n) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const bool bad = crc[i] != expected[i];
  if (mismatch) mismatch[i] = bad ? 1 : 0;
  if (bad && count) atomicAdd(count, 1u);
}

// Synthetic bytes: byte i of the stream = byte (i&7) of splitmix64(seed + ((i>>3)+1)*golden).
__device__ __forceinline__ uint64_t splitmix_mix(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

__global__ void fill_splitmix_kernel(uint8_t* __restrict__ dst, uint64_t nbytes, uint64_t seed, uint64_t stream_off) {
  // Requires dst 16-B aligned and stream_off % 16 == 0 (checked on the host).
  const uint64_t n16 = nbytes / 16;
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += stride) {
    const uint64_t word = (stream_off >> 3) + 2 * i;
    const uint64_t w0 = splitmix_mix(seed + (word + 1) * 0x9E3779B97F4A7C15ull);
    const uint64_t w1 = splitmix_mix(seed + (word + 2) * 0x9E3779B97F4A7C15ull);
    u32x4 v = {(uint32_t)w0, (uint32_t)(w0 >> 32), (uint32_t)w1, (uint32_t)(w1 >> 32)};
    reinterpret_cast<u32x4*>(dst)[i] = v;
  }
  if (blockIdx.x == 0 && threadIdx.x < (nbytes & 15)) {
    const uint64_t pos = stream_off + n16 * 16 + threadIdx.x;
    const uint64_t w = splitmix_mix(seed + ((pos >> 3) + 1) * 0x9E3779B97F4A7C15ull);
    dst[n16 * 16 + threadIdx.x] = (uint8_t)(w >> (8 * (pos & 7)));
  }
}

// ---------------------------------------------------------------- launchers
hipError_t launch_plan(const PlanArgs& a, hipStream_t s) {
  hipLaunchKernelGGL(crc32_plan_kernel, dim3(1), dim3(1024), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_tiles(const TilesArgs& a, int grid, int variant, hipStream_t s) {
  switch (variant) {
    case 0: hipLaunchKernelGGL((crc32_tiles_kernel<8, false>), dim3(grid), dim3(1024), 0, s, a); break;
    case 1: hipLaunchKernelGGL((crc32_tiles_kernel<8, true>), dim3(grid), dim3(1024), 0, s, a); break;
    case 2: hipLaunchKernelGGL((crc32_tiles_kernel<4, false>), dim3(grid), dim3(1024), 0, s, a); break;
    case 3: hipLaunchKernelGGL((crc32_tiles_kernel<16, false>), dim3(grid), dim3(1024), 0, s, a); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

hipError_t launch_verify(const uint32_t* crc, const uint32_t* expected, uint8_t* mismatch, uint32_t* count,
                         uint32_t n, hipStream_t s) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(crc32_verify_kernel, dim3((n + 255) / 256), dim3(256), 0, s, crc, expected, mismatch, count, n);
  return hipGetLastError();
}

hipError_t launch_fill(uint8_t* dst, uint64_t nbytes, uint64_t seed, uint64_t stream_off, hipStream_t s) {
  if (nbytes == 0) return hipSuccess;
  uint64_t n16 = nbytes / 16;
  uint64_t blocks = (n16 + 255) / 256;
  if (blocks > 65536) blocks = 65536;
  if (blocks == 0) blocks = 1;
  hipLaunchKernelGGL(fill_splitmix_kernel, dim3((uint32_t)blocks), dim3(256), 0, s, dst, nbytes, seed, stream_off);
  return hipGetLastError();
}

}  // namespace ambrycrc
