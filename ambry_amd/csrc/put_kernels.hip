// put_kernels.hip -- gfx950 kernels of the PUT-message write path (ambrycrc_serialize_puts_dev):
// the batch form of PutMessageFormatInputStream (PutMessageFormatInputStream.java:76-124) +
// MessageFormatInputStream.read* (MessageFormatInputStream.java:40-96), which Ambry's server runs
// per PUT, computing every record CRC while it streams the message out.
//
//   put_layout_kernel   one thread per message: header fields and record prefixes (byte stores,
//                       ~70 B per message), the copy jobs of the variable fields and the CRC jobs
//   gather_copy_kernel  byte-balanced copy of every job (HBM read + write bound): each wave owns
//                       an equal share of the concatenated job bytes; 16-B destination pieces are
//                       built from two aligned source loads and v_alignbyte_b32, so loads and
//                       stores stay coalesced whatever the source/destination misalignment
//   (plan + sweep)      the batch CRC kernels over the CRC jobs, in the output buffer
//   put_seal_kernel     one thread per CRC job: the big-endian 8-B trailer
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "crc32_kernels.h"
#include "crc_img.h"
#include "put_layout.h"
#include "record_fields.h"
#include "region_crc.h"

namespace ambrycrc {

typedef uint32_t u32x4p __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void put_layout_kernel(PutArgs a) {
  // The CRCs this kernel takes itself (the header's; copy-through's record-prefix seeds) run over
  // bytes it builds in registers, through LDS tables: not over bytes it just stored, read back
  // one dependent global load per byte.
  __shared__ uint32_t tbl[1024];
  if (a.gate && *a.gate == 0) return;  // grid-uniform
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint64_t m = a.m;
  const bool live = i < m;
  ambrycrc_put_desc d;
  PutLayout L;
  const bool ok = live && put_layout(d = a.desc[i], L);
  // copy mode: a message this short is the streamed kernels' (put_stream_kernel) and gets no jobs
  const bool streamed = a.stream_max && ok && L.length <= a.stream_max;
  if (a.clear_short) {  // the job path runs (a long message is present): the streamed ones' entries are empty
    if (streamed) {
      for (uint32_t k = 0; k < kPutSlots; ++k) {
        a.cp_len[k * m + i] = 0;
        a.cp_cost[k * m + i] = 0;
        a.crc_len[k * m + i] = 0;
        a.crc_off[k * m + i] = 0;
        a.crc_in[k * m + i] = 0;
      }
    }
    return;
  }
  bool hashes = a.copy_through || a.in_crc;  // kernel-uniform
  // with streaming, only a block holding a message for the job path hashes (every thread reaches the barrier)
  if (hashes && a.stream_max) hashes = __syncthreads_or(live && !streamed);
  if (hashes) {
    stage_slice_tables(tbl, a.img);
    __syncthreads();
  }
  if (!live) return;
  if (!ok) {  // the host checks descriptors it can see; a bad one here writes nothing
    for (uint32_t k = 0; k < kPutSlots; ++k) {
      a.cp_len[k * m + i] = 0;
      a.cp_cost[k * m + i] = 0;
      a.crc_len[k * m + i] = 0;
      a.crc_off[k * m + i] = 0;
      if (a.copy_through) a.crc_in[k * m + i] = 0;
    }
    if (a.msg_len) a.msg_len[i] = 0;
    return;
  }
  if (a.stream_max) {
    if (streamed) {  // its job entries: zeroed by the clear_short launch only if the job path runs
      if (a.msg_len) a.msg_len[i] = L.length;
      put_write_fixed(d, L, a.out + d.out_off);  // the gaps' bytes, which put_stream_kernel's edge pieces read
      return;
    }
    *a.big = 1u;  // a longer one: the job path runs (every writer stores the same word)
  }
  uint8_t* msg = a.out + d.out_off;
  put_write_fixed(d, L, msg);
  uint32_t head_crc = 0;
  if (hashes) {
    uint8_t h[32];
    const uint32_t hn = put_header_bytes(d, L, h);
    head_crc = crc_regs_lds(tbl, 0u, h, hn);
  }
  uint64_t fo[5];
  put_field_offsets(d, L, fo);
  const uint64_t src[5] = {d.key_src, d.enckey_src, d.props_src, d.usermeta_src, d.blob_src};
  // a transform's V5 re-encoding copies the stored payload; props_fix_kernel completes it
  const uint64_t props_copy = a.pfix && a.pfix[i].version ? a.pfix[i].stored_len : d.props_len;
  const uint64_t len[5] = {d.key_len, L.enc_rec ? (uint64_t)d.enckey_len : 0, props_copy, d.usermeta_len,
                           d.blob_len};
#pragma unroll
  for (uint32_t k = 0; k < kPutSlots; ++k) {
    const uint8_t* base = k == 4 ? a.blobs : a.fields;
    a.cp_src[k * m + i] = base ? (uint64_t)(uintptr_t)(base + src[k]) - a.src_base
                               : (a.copy_through ? (uint64_t)(uintptr_t)(msg + fo[k]) - a.src_base : 0);
    a.cp_dst[k * m + i] = d.out_off + fo[k];
    a.cp_len[k * m + i] = base || a.copy_through ? len[k] : 0;
    a.cp_cost[k * m + i] = base && len[k] ? len[k] + kCopyJobCost : 0;
    uint64_t off, ln;
    bool present;
    put_crc_job(L, k, &off, &ln, &present);
    a.crc_off[k * m + i] = d.out_off + off;
    a.crc_len[k * m + i] = present ? ln : 0;
    if (a.in_crc && present) {  // transform: every CRC known but the header's (hashed here)
      const uint32_t crc = k == 0 ? head_crc : a.in_crc[4 * i + k - 1];
      put_be64(msg + off + ln, (uint64_t)crc);
    }
    if (a.copy_through) {  // the batch's seeds: each record's prefix CRC; the header is hashed whole
      uint32_t seed = 0;
      if (k == 0) {
        put_be64(msg + ln, (uint64_t)head_crc);
      } else if (present) {
        uint8_t b[16];
        const uint32_t pl = put_prefix_bytes(d, k, b);
        seed = crc_regs_lds(tbl, 0u, b, pl);
      }
      a.crc_in[k * m + i] = seed;
    }
  }
  if (a.msg_len) a.msg_len[i] = L.length;
}

__global__ __launch_bounds__(256) void put_seal_kernel(PutArgs a) {
  const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= kPutSlots * a.m || (a.gate && *a.gate == 0)) return;
  if (a.copy_through && j < a.m) return;  // slot 0's job is the key; the layout kernel sealed the header
  const uint64_t len = a.crc_len[j];
  if (len == 0) return;  // absent encryption-key record (every present record has >= 6 bytes)
  put_be64(a.out + a.crc_off[j] + len, (uint64_t)a.crc[j]);
}

// ---------------------------------------------------------------- streamed small messages
// Pass 2 of copy-mode serialization for messages of at most kStreamPutMax bytes (put_stream_kernel,
// crc32_kernels.hip, wrote their bytes and the raw CRC of every 64-B output run): one thread per
// message computes the header CRC from the bytes it builds in registers and each record's CRC from the
// run sums (region::record_crc: the head and tail runs a record cuts re-read from the output), and
// writes the big-endian trailers -- the CRCs MessageFormatInputStream emits after each record
// (MessageFormatInputStream.java:85-93; PutMessageFormatInputStream.java:76-124). Two blocks per CU, as
// region_msg_kernel, so a thread's lines stay in L2 between its dependent reads.
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(AMBRY_REGION_WPE))) void put_stream_seal_kernel(
    StreamPutArgs a) {
  __shared__ uint32_t tbl[1024];
  __shared__ uint32_t nib[region::kNibTotal];
  __shared__ uint32_t hm[kRegAuxWords], bt[kRegByteWords], un[kRegUnWords];
  stage_slice_tables(tbl, a.img);
  region::stage_nib(nib, a.img);
  region::stage_aux(hm, bt, un, a.img);
  __syncthreads();
  const region::Aux aux{hm, bt, un};
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < a.m; i += (uint64_t)gridDim.x * blockDim.x) {
    const ambrycrc_put_desc d = a.desc[i];
    PutLayout L;
    if (!put_layout(d, L) || L.length > kStreamPutMax) continue;
    const uint64_t m0 = a.oreg0 + d.out_off;
    uint8_t* msg = a.obase + m0;
    // message i's run slots, addressed by base-relative run index (record_crc's rk[k])
    const uint32_t* rk = reinterpret_cast<const uint32_t*>(
        reinterpret_cast<uintptr_t>(a.rk + kRunPad + i * kStreamPutRuns) - ((m0 >> 6) << 2));
    uint8_t h[32];
    const uint32_t hn = put_header_bytes(d, L, h);
    put_be64(msg + hn, (uint64_t)crc_regs_lds(tbl, 0u, h, hn));
#pragma unroll 1
    for (uint32_t k = 1; k < kPutSlots; ++k) {
      uint64_t off, ln;
      bool present;
      put_crc_job(L, k, &off, &ln, &present);
      if (!present) continue;
      const uint32_t c = region::record_crc(region::TabC{tbl}, nib, a.obase, rk, m0 + off, ln, aux);
      put_be64(msg + off + ln, (uint64_t)c);
    }
  }
}

hipError_t launch_put_stream_seal(const StreamPutArgs& a, int num_cu, hipStream_t s) {
  if (a.m == 0) return hipSuccess;
  uint64_t blocks = (a.m + 255) / 256;
  if (blocks > (uint64_t)num_cu * AMBRY_SEAL_BPC) blocks = (uint64_t)num_cu * AMBRY_SEAL_BPC;
  hipLaunchKernelGGL(put_stream_seal_kernel, dim3((uint32_t)blocks), dim3(256), 0, s, a);
  return hipGetLastError();
}

// ---------------------------------------------------------------- gather copy
__device__ __forceinline__ uint64_t rl64(uint64_t v, uint32_t lane) {
  const uint32_t lo = __builtin_amdgcn_readlane((uint32_t)v, lane);
  const uint32_t hi = __builtin_amdgcn_readlane((uint32_t)(v >> 32), lane);
  return ((uint64_t)hi << 32) | lo;
}

// Largest c in [0, n) with start[c] <= g (start nondecreasing, start[0] = 0): 64-ary search.
__device__ __forceinline__ uint32_t find_job(const uint64_t* __restrict__ start, uint32_t n, uint64_t g,
                                             uint32_t lane) {
  uint32_t lo = 0, hi = n;
  while (hi - lo > 1) {
    const uint32_t step = (hi - lo + 63) / 64;
    const uint32_t idx = lo + lane * step;
    const uint64_t m = __ballot(idx < hi && start[idx] <= g);
    const uint32_t last = 63u - (uint32_t)__builtin_clzll(m);
    const uint32_t nhi = lo + (last + 1) * step;
    lo = lo + last * step;
    hi = nhi < hi ? nhi : hi;
  }
  return lo;
}

// Dword k of bytes [4Q + r, 4Q + r + 16) of the 32-byte concatenation a||b (little endian).
template <int Q>
__device__ __forceinline__ u32x4p shift_pair(const u32x4p& a, const u32x4p& b, uint32_t r) {
  const uint32_t w[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
  u32x4p o;
  if (r == 0) {
    o.x = w[Q];
    o.y = w[Q + 1];
    o.z = w[Q + 2];
    o.w = w[Q + 3];
  } else {
    o.x = __builtin_amdgcn_alignbyte(w[Q + 1], w[Q], r);
    o.y = __builtin_amdgcn_alignbyte(w[Q + 2], w[Q + 1], r);
    o.z = __builtin_amdgcn_alignbyte(w[Q + 3], w[Q + 2], r);
    o.w = __builtin_amdgcn_alignbyte(w[Q + 4], w[Q + 3], r);
  }
  return o;
}

// Copies n16 16-B pieces to the 16-B aligned dst from src (any alignment: shift = 4Q + r),
// lane-strided, 4 pieces per lane in flight. The second aligned source block of a piece holds
// bytes the piece needs whenever shift > 0, so every load touches the source range.
template <int Q>
__device__ __forceinline__ void copy_pieces(uint8_t* __restrict__ dst, const uint8_t* __restrict__ src, uint64_t n16,
                                            uint32_t r, uint32_t lane) {
  const uint32_t shift = 4 * Q + r;
  const u32x4p* s0 = reinterpret_cast<const u32x4p*>(src - shift);
  u32x4p* d0 = reinterpret_cast<u32x4p*>(dst);
  constexpr int U = 4;
  uint64_t p = lane;
  for (; p + 64 * (U - 1) < n16; p += 64 * U) {
    u32x4p a[U], b[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      a[u] = __builtin_nontemporal_load(s0 + p + 64 * u);
      b[u] = shift ? __builtin_nontemporal_load(s0 + p + 64 * u + 1) : u32x4p{0u, 0u, 0u, 0u};
    }
#pragma unroll
    for (int u = 0; u < U; ++u) __builtin_nontemporal_store(shift_pair<Q>(a[u], b[u], r), d0 + p + 64 * u);
  }
  for (; p < n16; p += 64) {
    const u32x4p a = __builtin_nontemporal_load(s0 + p);
    const u32x4p b = shift ? __builtin_nontemporal_load(s0 + p + 1) : u32x4p{0u, 0u, 0u, 0u};
    __builtin_nontemporal_store(shift_pair<Q>(a, b, r), d0 + p);
  }
}

// One wave copies n bytes src -> dst (wave-uniform arguments).
__device__ __forceinline__ void copy_range(uint8_t* __restrict__ dst, const uint8_t* __restrict__ src, uint64_t n,
                                           uint32_t lane) {
  const uint64_t head0 = (16 - ((uintptr_t)dst & 15)) & 15;
  const uint64_t head = head0 < n ? head0 : n;
  if (lane < head) dst[lane] = src[lane];
  const uint64_t body = n - head;
  const uint64_t n16 = body >> 4;
  uint8_t* d1 = dst + head;
  const uint8_t* s1 = src + head;
  if (n16) {
    const uint32_t shift = (uint32_t)((uintptr_t)s1 & 15);
    switch (shift >> 2) {
      case 0: copy_pieces<0>(d1, s1, n16, shift & 3, lane); break;
      case 1: copy_pieces<1>(d1, s1, n16, shift & 3, lane); break;
      case 2: copy_pieces<2>(d1, s1, n16, shift & 3, lane); break;
      default: copy_pieces<3>(d1, s1, n16, shift & 3, lane); break;
    }
  }
  const uint64_t t = body & 15;
  if (lane < t) d1[16 * n16 + lane] = s1[16 * n16 + lane];
}

// Persistent, cost-balanced: wave w takes [w*S, (w+1)*S) of the jobs' concatenated costs (start =
// exclusive scan of len + kCopyJobCost, from the plan kernel); job j's bytes are the first len[j]
// units of its cost range, so every byte is copied by exactly one wave. Descriptors 64 at a time.
__global__ __launch_bounds__(256) void gather_copy_kernel(CopyArgs a) {
  if (a.gate && *a.gate == 0) return;  // uniform
  const uint32_t lane = threadIdx.x & 63u;
  const uint64_t nwaves = (uint64_t)gridDim.x * (blockDim.x >> 6);
  const uint32_t wave = __builtin_amdgcn_readfirstlane((threadIdx.x >> 6) * gridDim.x + blockIdx.x);
  const uint64_t total = a.start[a.n];
  uint64_t S = (total + nwaves - 1) / nwaves;
  S = (S + 255) & ~uint64_t(255);
  S = S < 4096 ? 4096 : S;
  const uint64_t g0 = (uint64_t)wave * S;
  if (g0 >= total) return;
  const uint64_t g1 = g0 + S < total ? g0 + S : total;
  uint32_t c = __builtin_amdgcn_readfirstlane(find_job(a.start, a.n, g0, lane));
  while (c < a.n) {
    const uint32_t cnt = a.n - c < 64u ? a.n - c : 64u;
    uint64_t w_st = ~0ull, w_len = 0, w_src = 0, w_dst = 0;
    if (lane < cnt) {
      w_st = a.start[c + lane];
      w_len = a.len[c + lane];
      w_src = a.src[c + lane];
      w_dst = a.dst_off[c + lane];
    }
    bool work = false;
    for (uint32_t j = 0; j < cnt; ++j) {
      const uint64_t st = rl64(w_st, j);
      if (st >= g1) return;
      const uint64_t len = rl64(w_len, j);
      if (len == 0) continue;
      work = true;
      const uint64_t r0 = g0 > st ? g0 - st : 0;
      const uint64_t r1 = g1 - st < len ? g1 - st : len;
      if (r0 < r1)
        copy_range(a.dst + rl64(w_dst, j) + r0,
                   reinterpret_cast<const uint8_t*>((uintptr_t)rl64(w_src, j)) + r0, r1 - r0, lane);
    }
    // A window of empty jobs (e.g. the encryption-key slot of messages without one: cost 0, all
    // at one start) may be the head of a long run; jump to its end instead of walking it 64 at a time.
    uint32_t next = c + cnt;
    if (!work && next < a.n) {
      const uint32_t far = __builtin_amdgcn_readfirstlane(find_job(a.start, a.n, rl64(w_st, cnt - 1), lane));
      next = far > next ? far : next;
    }
    c = next;
  }
}

hipError_t launch_put_layout(const PutArgs& a, hipStream_t s) {
  if (a.m == 0) return hipSuccess;
  hipLaunchKernelGGL(put_layout_kernel, dim3((uint32_t)((a.m + 255) / 256)), dim3(256), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_put_seal(const PutArgs& a, hipStream_t s) {
  if (a.m == 0) return hipSuccess;
  hipLaunchKernelGGL(put_seal_kernel, dim3((uint32_t)((kPutSlots * a.m + 255) / 256)), dim3(256), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_gather_copy(const CopyArgs& a, int grid, hipStream_t s) {
  if (a.n == 0) return hipSuccess;
  hipLaunchKernelGGL(gather_copy_kernel, dim3(grid), dim3(256), 0, s, a);
  return hipGetLastError();
}

}  // namespace ambrycrc
