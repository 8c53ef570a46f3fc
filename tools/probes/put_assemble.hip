// put_assemble.hip -- A/B probe, not in the product library: whole-message
// assembly of the serialize copy mode. Built, parity-green, and measured 1.5-1.7x slower than the
// layout + copy-through sweep + seal path (instruction-bound at ~3,500 wave instructions per
// message), so round 5 moved it here from csrc/put_kernels.hip. tools/ab_build.sh compiles it into
// A/B builds with -DAMBRY_AB_PUT_ASSEMBLE -DAMBRY_AB_PROBE_BUILD, appended to put_kernels.hip (it
// uses that file's includes and shift_pair); AMBRYCRC_ASM_MAX (<= 6144) at init then turns it on.
#ifndef AMBRY_AB_PUT_ASSEMBLE
#error "A/B only: tools/ab_build.sh appends it to put_kernels.hip with -DAMBRY_AB_PUT_ASSEMBLE -DAMBRY_AB_PROBE_BUILD"
#endif

namespace ambrycrc {

// ---------------------------------------------------------------- whole-message assembly
// put_assemble_kernel (copy mode with both field buffers; messages of at most kAsmMaxBytes): a wave
// per message builds it in an LDS image laid on the output's 16-B grid -- each data field's pieces
// from its source (two aligned 16-B loads and v_alignbyte_b32 per piece, bytes outside the field
// masked), then the header and record prefixes, byte by byte across lanes -- hashes every record
// from the image's pieces, writes the trailers into the image and stores the message as 16-B
// pieces: every 128-B line inside the message in one wave's stores, the two lines it shares with
// its neighbours in the same instant as theirs (adjacent waves take adjacent messages). Round 3's
// path wrote the header and prefixes, the fields and the trailers from three kernels hundreds of
// microseconds apart: ~7 partial lines per message written back half-filled (1.114x traffic).
//
// A record [s, e): piece p holds message bytes [16p - a0, 16p - a0 + 16) (a0: the message's start
// mod 16). Lane l's raw CRC of its piece (bytes outside [s, e) zero, the first four XORed with
// 0xFF: zlib's initial register) is folded over its pieces l, l + 64, ... up to q (the piece
// holding e - 1) by x^(8*1024); the lanes are rotated so that lane (q mod 64) lands last, and a DPP
// tree (x^(8*16*2^k)) gives the register at the end of piece q, un-shifted by its d = 16(q + 1) -
// a0 - e < 16 bytes past e (x^(-8*2^k) sets). Model: tests/kernel_model.py assembly_crc.
namespace asmk {
constexpr uint32_t kSets = 11;  // nibble sets in LDS: TREE[0..5], FOLD, x^(-8*2^k) k = 0..3
constexpr uint32_t kTree0 = 0, kFold = 6, kInv0 = 7;
constexpr uint32_t kChunks = (kAsmMaxBytes + 15 + 1023) / 1024;  // 1 KiB chunks of a message's pieces
constexpr uint32_t kImgBytes = kChunks * 1024;
constexpr uint32_t kWaves = 4;
}  // namespace asmk

// v (bytes [sh, sh + 16) of w0 || w1), sh wave-uniform.
__device__ __forceinline__ u32x4p funnel16(const u32x4p& w0, const u32x4p& w1, uint32_t sh) {
  switch (sh >> 2) {
    case 0: return shift_pair<0>(w0, w1, sh & 3u);
    case 1: return shift_pair<1>(w0, w1, sh & 3u);
    case 2: return shift_pair<2>(w0, w1, sh & 3u);
    default: return shift_pair<3>(w0, w1, sh & 3u);
  }
}

// Bytes of piece-relative range [lo, hi) kept (others zero).
__device__ __forceinline__ u32x4p keep_range(u32x4p v, int lo, int hi) {
  v.x &= region::keep_ge(lo) & region::keep_lt(hi);
  v.y &= region::keep_ge(lo - 4) & region::keep_lt(hi - 4);
  v.z &= region::keep_ge(lo - 8) & region::keep_lt(hi - 8);
  v.w &= region::keep_ge(lo - 12) & region::keep_lt(hi - 12);
  return v;
}

__global__ __launch_bounds__(256) void put_assemble_kernel(PutArgs a) {
  __shared__ uint32_t tbl[1024];
  __shared__ uint32_t nib[asmk::kSets * region::kNibWords];
  __shared__ __attribute__((aligned(16))) uint8_t image[asmk::kWaves][asmk::kImgBytes];
  stage_slice_tables(tbl, a.img);
  for (uint32_t i = threadIdx.x; i < asmk::kSets * region::kNibWords; i += blockDim.x) {
    const uint32_t set = i / region::kNibWords, w = i % region::kNibWords;
    const uint32_t byte = set < asmk::kFold ? kNibBase + kTreeOff + kNibSetBytes * set
                          : set == asmk::kFold ? kNibBase + kFoldOff
                                               : kImgInvOff + kNibSetBytes * (set - asmk::kInv0);
    nib[i] = a.img[byte / 4 + w];
  }
  __syncthreads();
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  uint8_t* img8 = image[wv];
  const region::TabC tc{tbl};
  const uint64_t nwaves = (uint64_t)gridDim.x * asmk::kWaves;
  bool big = false;
  for (uint64_t i = (uint64_t)blockIdx.x * asmk::kWaves + wv; i < a.m; i += nwaves) {
    const ambrycrc_put_desc d = a.desc[i];
    PutLayout L;
    if (!put_layout(d, L)) {  // nothing written (as put_layout_kernel)
      if (lane == 0 && a.msg_len) a.msg_len[i] = 0;
      continue;
    }
    if (L.length > a.asm_max) {  // the job path's
      big = true;
      continue;
    }
    uint8_t* ob = a.out + d.out_off;
    const int32_t a0 = (int32_t)((uintptr_t)ob & 15u);
    const int32_t len = (int32_t)L.length;
    const uint32_t npieces = (uint32_t)(len + a0 + 15) >> 4;
    uint64_t fo[5];
    put_field_offsets(d, L, fo);
    const uint32_t flen[5] = {d.key_len, L.enc_rec ? (uint32_t)d.enckey_len : 0u, d.props_len, d.usermeta_len,
                              (uint32_t)d.blob_len};
    const uint64_t fsrc[5] = {d.key_src, d.enckey_src, d.props_src, d.usermeta_src, d.blob_src};
    // 1. the data fields' pieces, into registers and the image. Field k's bytes for the piece at
    // message position P start at offset x = P - ds + (src & 15) from its first aligned block:
    // the blocks at x - sh and x - sh + 16 (sh = x mod 16, the same for every piece), clamped to
    // the field's own blocks (a clamped block only feeds bytes outside the field, masked).
    const uint8_t* blk[5];
    int32_t mis[5], last[5];
    uint32_t sh[5];
#pragma unroll
    for (uint32_t k = 0; k < 5; ++k) {
      const uint8_t* base = (k == 4 ? a.blobs : a.fields) + fsrc[k];
      mis[k] = (int32_t)((uintptr_t)base & 15u);
      blk[k] = base - mis[k];
      last[k] = (mis[k] + (int32_t)flen[k] - 1) & ~15;
      sh[k] = (uint32_t)(mis[k] - (int32_t)fo[k] - a0) & 15u;
    }
    u32x4p pc[asmk::kChunks];
#pragma unroll
    for (uint32_t u = 0; u < asmk::kChunks; ++u) {
      pc[u] = u32x4p{0u, 0u, 0u, 0u};
      const int32_t c0 = (int32_t)(1024 * u) - a0;  // the chunk's message span [c0, c0 + 1024)
      if (c0 >= len) continue;
      const int32_t P = c0 + 16 * (int32_t)lane;
#pragma unroll
      for (uint32_t k = 0; k < 5; ++k) {
        const int32_t ds = (int32_t)fo[k], de = ds + (int32_t)flen[k];
        if (flen[k] == 0 || de <= c0 || ds >= c0 + 1024) continue;  // (wave-uniform)
        const int lo = ds - P, hi = de - P;
        if (lo < 16 && hi > 0) {
          const int32_t x0 = P - ds + mis[k] - (int32_t)sh[k];
          const int32_t b0 = min(max(x0, 0), last[k]), b1 = min(max(x0 + 16, 0), last[k]);
          const u32x4p w0 = *reinterpret_cast<const u32x4p*>(blk[k] + b0);
          const u32x4p w1 = *reinterpret_cast<const u32x4p*>(blk[k] + b1);
          u32x4p v = funnel16(w0, w1, sh[k]);
          if (lo > 0 || hi < 16) v = keep_range(v, lo, hi);  // the field's first / last piece
          pc[u] |= v;
        }
      }
    }
#pragma unroll
    for (uint32_t u = 0; u < asmk::kChunks; ++u)  // (after every chunk's loads are issued)
      if ((int32_t)(1024 * u) - a0 < len && lane + 64 * u < npieces)
        *reinterpret_cast<u32x4p*>(img8 + 16 * (lane + 64 * u)) = pc[u];
    // 2. header and record prefixes into the image, lane b taking byte b of each big-endian field
    auto put_be = [&](int32_t pos, uint32_t width, uint64_t v) {
      if (lane < width) img8[pos + a0 + (int32_t)lane] = (uint8_t)(v >> (8 * (width - 1 - lane)));
    };
    uint8_t h[32];
    const uint32_t hn = put_header_bytes(d, L, h);
    const uint32_t hcrc = crc_regs_lds(tbl, 0u, h, hn);
    {
      uint32_t hw[8];
#pragma unroll
      for (int q = 0; q < 8; ++q)
        hw[q] = (uint32_t)h[4 * q] | (uint32_t)h[4 * q + 1] << 8 | (uint32_t)h[4 * q + 2] << 16 |
                (uint32_t)h[4 * q + 3] << 24;
      uint32_t w = hw[0];
#pragma unroll
      for (int q = 1; q < 8; ++q) w = (lane >> 2) == (uint32_t)q ? hw[q] : w;
      if (lane < hn) img8[a0 + (int32_t)lane] = (uint8_t)(w >> (8 * (lane & 3u)));
    }
    put_be((int32_t)hn, 8, hcrc);
    if (L.enc_rec) {
      put_be(L.enc_rel, 2, 1);
      put_be(L.enc_rel + 2, 4, (uint32_t)d.enckey_len);
    }
    put_be(L.bp_rel, 2, 1);
    put_be(L.um_rel, 2, 1);
    put_be(L.um_rel + 2, 4, d.usermeta_len);
    put_be(L.blob_rel, 2, 3);
    put_be(L.blob_rel + 2, 2, (uint32_t)(uint16_t)d.blob_type);
    put_be(L.blob_rel + 4, 1, d.compressed ? 1u : 0u);
    put_be(L.blob_rel + 5, 8, d.blob_len);
    // the pieces back with their prefixes (a wave's LDS operations complete in order)
#pragma unroll
    for (uint32_t u = 0; u < asmk::kChunks; ++u)
      if ((int32_t)(1024 * u) - a0 < len && lane + 64 * u < npieces)
        pc[u] = *reinterpret_cast<const u32x4p*>(img8 + 16 * (lane + 64 * u));
    // 3. the record CRCs (encryption key, properties, user metadata, blob) and their trailers
#pragma unroll 1
    for (uint32_t k = 1; k < kPutSlots; ++k) {
      if (k == 1 && !L.enc_rec) continue;
      const int32_t s = put_record_rel(L, k), e = (int32_t)fo[k] + (int32_t)flen[k];
      const int32_t rlen = e - s;
      const int ni = rlen < 4 ? rlen : 4;  // zlib's initial register over the first bytes
      const uint32_t q = (uint32_t)(e - 1 + a0) >> 4, p0 = (uint32_t)(s + a0) >> 4;
      const uint32_t dsh = 16 * (q + 1) - (uint32_t)a0 - (uint32_t)e;
      uint32_t acc = 0;
#pragma unroll
      for (uint32_t u = 0; u < asmk::kChunks; ++u) {
        if (64 * u > q || 64 * u + 63 < p0) continue;  // (wave-uniform)
        const uint32_t p = lane + 64 * u;
        if (p <= q) {
          const int32_t P = 16 * (int32_t)p - a0;
          const int lo = s - P, hi = e - P;
          u32x4p v = pc[u];
          if (lo > 0 || hi < 16) v = keep_range(v, lo, hi);  // the record's first / last piece
          if (lo > -4 && lo < 16) {  // its first bytes
            v.x ^= region::keep_ge(lo) & region::keep_lt(lo + ni);
            v.y ^= region::keep_ge(lo - 4) & region::keep_lt(lo + ni - 4);
            v.z ^= region::keep_ge(lo - 8) & region::keep_lt(lo + ni - 8);
            v.w ^= region::keep_ge(lo - 12) & region::keep_lt(lo + ni - 12);
          }
          uint32_t c = tc.step4(v.x);
          c = tc.step4(c ^ v.y);
          c = tc.step4(c ^ v.z);
          c = tc.step4(c ^ v.w);
          acc = region::nmul(nib, acc, asmk::kFold) ^ c;
        }
      }
      // lane l's fold ends (q - l) mod 64 pieces before q: rotate it to virtual lane 63 - that.
      // A record of n < 64 pieces then sits in the top n lanes: levels 2^k >= n add only zeros.
      uint32_t t = (uint32_t)__shfl((int)acc, (int)((lane + q + 1) & 63u));
      const uint32_t nrec = q - p0 + 1;
      if (1u < nrec) {
        const uint32_t pt = region::left_partner<0>(t);
        if (lane & 1u) t ^= region::nmul(nib, pt, asmk::kTree0 + 0);
      }
      if (2u < nrec) {
        const uint32_t pt = region::left_partner<1>(t);
        if (lane & 2u) t ^= region::nmul(nib, pt, asmk::kTree0 + 1);
      }
      if (4u < nrec) {
        const uint32_t pt = region::left_partner<2>(t);
        if (lane & 4u) t ^= region::nmul(nib, pt, asmk::kTree0 + 2);
      }
      if (8u < nrec) {
        const uint32_t pt = region::left_partner<3>(t);
        if (lane & 8u) t ^= region::nmul(nib, pt, asmk::kTree0 + 3);
      }
      if (16u < nrec) {
        const uint32_t pt = region::left_partner<4>(t);
        if (lane & 16u) t ^= region::nmul(nib, pt, asmk::kTree0 + 4);
      }
      if (32u < nrec) {
        const uint32_t pt = region::left_partner<5>(t);
        if (lane & 32u) t ^= region::nmul(nib, pt, asmk::kTree0 + 5);
      }
      uint32_t V = __builtin_amdgcn_readlane(t, 63);
#pragma unroll
      for (uint32_t b = 0; b < 4; ++b)
        if (dsh & (1u << b)) V = region::nmul(nib, V, asmk::kInv0 + b);
      if (rlen < 4) V ^= 0xFFFFFFFFu >> (8 * rlen);
      put_be(e, 8, (uint64_t)~V);
    }
    // 4. the message out: every piece inside it as one 16-B store; the bytes of the pieces it shares
    // with what lies before / after it (a neighbour, a gap) lane by lane
    const int32_t head = a0 ? min(16 - a0, len) : 0;                // bytes [0, head)
    const int32_t tail0 = max(head, ((len + a0) & ~15) - a0);       // bytes [tail0, len)
#pragma unroll
    for (uint32_t u = 0; u < asmk::kChunks; ++u) {
      const uint32_t p = lane + 64 * u;
      const int32_t P = 16 * (int32_t)p - a0;
      if ((int32_t)(1024 * u) - a0 >= len) continue;  // (wave-uniform)
      if (P >= 0 && P + 16 <= len)
        *reinterpret_cast<u32x4p*>(ob + P) = *reinterpret_cast<const u32x4p*>(img8 + 16 * p);
    }
    if ((int32_t)lane < head) ob[lane] = img8[a0 + (int32_t)lane];
    if (tail0 + (int32_t)lane < len) ob[tail0 + (int32_t)lane] = img8[a0 + tail0 + (int32_t)lane];
    if (lane == 0 && a.msg_len) a.msg_len[i] = L.length;
  }
  if (__ballot(big) && lane == 0) atomicOr(a.big, 1u);  // one per wave: many waves, one word
}

hipError_t launch_put_assemble(const PutArgs& a, int num_cu, hipStream_t s) {
  if (a.m == 0) return hipSuccess;
  uint64_t blocks = (a.m + asmk::kWaves - 1) / asmk::kWaves;
  if (blocks > (uint64_t)num_cu * 4) blocks = (uint64_t)num_cu * 4;
  hipLaunchKernelGGL(put_assemble_kernel, dim3((uint32_t)blocks), dim3(64 * asmk::kWaves), 0, s, a);
  return hipGetLastError();
}

}  // namespace ambrycrc
