// message_kernels.hip -- batched verify of Ambry PUT / update messages in a log region
// (SURVEY.md §8f next #1): the GPU form of deserializeBlobAll's CRC checks
// (ambry-messageformat/.../MessageFormatRecord.java:257-303), BlobStoreRecovery's
// per-message verification (ambry-store/.../BlobStoreRecovery.java:43-110) and
// ValidatingTransformer's replication check (ValidatingTransformer.java:46-104).
//
// Pipeline (all on the caller's stream):
//   msg_parse_kernel   one thread per message: header version, header CRC (<= 32 B,
//                      slice-by-4 through LDS tables), header constraints, and up to five record
//                      CRC jobs (enc key, properties, update, user metadata, blob) =
//                      [record start, record end - 8) with the stored big-endian CRC; job
//                      k*m + i is slot k of message i (slot-major: coalesced stores). The
//                      stored CRC of a record the group phase takes whole (<= inline_max)
//                      is left to the sweep, which streams that line anyway
//   plan + sweep       the batch CRC engine over the 5m jobs (crc32_kernels.hip)
//   msg_reduce_kernel  per-message status bits: computed CRC vs expected, per record slot
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/ambrycrc.h"
#include "crc32_kernels.h"
#include "crc32_layout.h"
#include "crc_img.h"
#include "put_layout.h"
#include "msg_parse.h"
#include "record_fields.h"
#include "region_crc.h"

namespace ambrycrc {

__device__ __forceinline__ void transform_describe(const TransformArgs& a, uint64_t i, uint32_t st0,
                                                   const PropsFields* pre = nullptr);


// DESC: the transform's speculative pass -- describe each message right after parsing it, from
// the header and record heads this thread just loaded (transform_describe's reads hit the cache).
// Grid: AMBRY_PARSE_BPC 256-thread blocks per CU, each thread looping over messages (0 = one
// thread per message); fewer messages in flight keep a thread's lines in L2 between its dependent
// reads (as region_msg_kernel's grid cap). A/B, the transform's fused parse over 262,144 4 KiB-blob
// messages: one thread per message 99.1 us, 2 blocks per CU 95.8, 4 blocks 99.0.
template <bool DESC>
__global__ __launch_bounds__(256) void msg_parse_kernel(MsgArgs a, TransformArgs t) {
  if (a.gate && *a.gate == 0) return;  // uniform
  __shared__ uint32_t tbl[1024];
  __shared__ uint32_t pwin[256 * kPropsSlotWords];
  stage_slice_tables(tbl, a.img);
  __syncthreads();
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < a.m; i += (uint64_t)gridDim.x * blockDim.x) {
    PropsFields pf;
    bool pf_ok = false;
    const uint64_t off = a.msg_off[i];
    const bool in_region = off <= a.region_len;
    const uint64_t rem = in_region ? a.region_len - off : 0;
    const uint8_t* p = a.region + (in_region ? off : 0);
    const HeaderWords hw = load_header(p, rem);
    MsgParse r;
    parse_message<DESC>(off, in_region, rem, p, hw, tbl, pwin + threadIdx.x * kPropsSlotWords, a.inline_max, r, pf,
                        pf_ok);
    // Jobs are slot-major (job k*m + i = slot k of message i), so each slot's store below is
    // one coalesced wave store; every slot is written exactly once.
#pragma unroll
    for (int k = 0; k < kMsgSlots; ++k) {
      a.job_off[(uint64_t)k * a.m + i] = r.jo[k];
      a.job_len[(uint64_t)k * a.m + i] = r.jl[k];
      a.expected[(uint64_t)k * a.m + i] = r.ex[k];
    }
    a.status[i] = r.status;
    if (a.msg_end) a.msg_end[i] = r.end ? off + r.end : 0;
    if constexpr (DESC) transform_describe(t, i, r.status, pf_ok ? &pf : nullptr);
  }
}

static uint32_t parse_blocks(uint64_t m) {
  uint64_t blocks = (m + 255) / 256;
  int dev = 0, cu = 0;
  if (AMBRY_PARSE_BPC > 0 && hipGetDevice(&dev) == hipSuccess &&
      hipDeviceGetAttribute(&cu, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && cu > 0 &&
      blocks > (uint64_t)cu * AMBRY_PARSE_BPC)
    blocks = (uint64_t)cu * AMBRY_PARSE_BPC;
  return (uint32_t)blocks;
}

// Region mode, pass 2: one thread per message parses it as msg_parse_kernel does
// (every stored CRC read here), assembles each record's CRC from the run sums of pass 1
// (region_crc.h) and writes the message's status: parse, CRC jobs, plan, sweep and reduce in one
// kernel, with no job arrays.
// Grid: AMBRY_REGION_BPC 256-thread blocks per CU (8 waves), each thread looping over messages,
// registers allowed for 2 waves per SIMD (AMBRY_REGION_WPE). Fewer messages in flight keep each
// thread's header / record-head lines in L2 until its own end-run reads (A/B, 4 KiB-blob messages:
// one thread per message at 16 waves per CU 120.1 us; 2 blocks per CU 104.9, with WPE 2 102.7; 3
// blocks 109.5; 1 block 135.4). 0 = one thread per message.
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(AMBRY_REGION_WPE))) void region_msg_kernel(
    MsgArgs a, RegionArgs g) {
  __shared__ uint32_t tbl[1024];
  __shared__ uint32_t pwin[256 * kPropsSlotWords];
  __shared__ uint32_t nib[region::kNibTotal];
  __shared__ uint32_t hm[kRegAuxWords], bt[kRegByteWords], un[kRegUnWords];
  // Long records (more than region::kLongRuns runs: a 4 MiB blob among small messages) are queued
  // per wave and taken by the whole wave after its messages (record_crc_runs_wave): one thread
  // walking 65,536 run sums would hold the kernel for milliseconds.
  constexpr uint32_t kLongQ = 32;
  __shared__ uint64_t lq_jo[4][kLongQ], lq_i[4][kLongQ];
  __shared__ uint32_t lq_jl[4][kLongQ], lq_ex[4][kLongQ], lq_bit[4][kLongQ], lq_n[4];
  stage_slice_tables(tbl, a.img);
  region::stage_nib(nib, a.img);
  region::stage_aux(hm, bt, un, a.img);
  if (threadIdx.x < 4) lq_n[threadIdx.x] = 0;
  __syncthreads();
  const region::Aux aux{hm, bt, un};
  const uint32_t wv = threadIdx.x >> 6, lane = threadIdx.x & 63u;
  uint32_t* slot = pwin + threadIdx.x * kPropsSlotWords;
  const uint32_t* rk = g.rk + kRunPad;
  // Grid-stride over the messages (a grid of one thread per message unless capped; no barrier
  // below, so threads leave the loop independently).
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < a.m; i += (uint64_t)gridDim.x * blockDim.x) {
    PropsFields pf;
    bool pf_ok = false;
    const uint64_t off = a.msg_off[i];
    const bool in_region = off <= a.region_len;
    const uint64_t rem = in_region ? a.region_len - off : 0;
    const uint8_t* p = a.region + (in_region ? off : 0);
    const HeaderWords hw = load_header(p, rem);
    uint32_t status = 0;
    uint64_t end;
    // One record's CRC from the run sums (long records to region_long_kernel's list, else to the
    // wave's queue), its bit into `status` on a mismatch.
    auto take = [&](int k, uint64_t jo, uint64_t jl, uint32_t ex) {
      const uint64_t pa = g.reg0 + jo;
      if (jl && (int64_t)((((pa + jl + 63) & ~uint64_t(63)) - (pa & ~uint64_t(63))) >> 6) > region::kLongRuns) {
        // to region_long_kernel (the whole grid takes it, piece by piece) unless the list is full
        if (g.lng.ctr && region::list_long(g.lng, pa, jl, ex, i, AMBRYCRC_MSG_ENCKEY_CRC << k)) return;
        const uint32_t at = atomicAdd(&lq_n[wv], 1u);
        if (at < kLongQ) {  // the wave's, after the loop (its bit ORed into the status then)
          lq_jo[wv][at] = pa;
          lq_i[wv][at] = i;
          lq_jl[wv][at] = (uint32_t)jl;
          lq_ex[wv][at] = ex;
          lq_bit[wv][at] = AMBRYCRC_MSG_ENCKEY_CRC << k;
          return;
        }
      }
#if AMBRY_REGION_PROBE == 1
      const uint32_t c = ex;
#else
      const uint32_t c = jl ? region::record_crc(region::TabC{tbl}, nib, g.base, rk, pa, jl, aux) : 0u;
#endif
      if (c != ex) status |= AMBRYCRC_MSG_ENCKEY_CRC << k;
    };
    {
      MsgParse r;
      parse_message<false>(off, in_region, rem, p, hw, tbl, slot, 0, r, pf, pf_ok);
      // The jobs go to this thread's LDS slot (the properties window is done with), so the five
      // descriptors do not stay live in VGPRs across the record CRCs: 4 words per slot, job start
      // relative to the message (records < 4 GiB: an int32 size field, blobs <= Integer.MAX_VALUE).
#pragma unroll
      for (int k = 0; k < kMsgSlots; ++k) {
        slot[4 * k] = (uint32_t)(r.jo[k] - off);
        slot[4 * k + 1] = (uint32_t)((r.jo[k] - off) >> 32);
        slot[4 * k + 2] = (uint32_t)r.jl[k];
        slot[4 * k + 3] = r.ex[k];
      }
      status = r.status;
      end = r.end;
    }
    static_assert(4 * kMsgSlots <= kPropsSlotWords, "job slots fit the properties window");
    for (int k = 0; k < kMsgSlots; ++k)
      take(k, off + ((uint64_t)slot[4 * k + 1] << 32 | slot[4 * k]), slot[4 * k + 2], slot[4 * k + 3]);
    a.status[i] = status;
    if (a.msg_end) a.msg_end[i] = end ? off + end : 0;
  }
  // the waves' long records (the loop above ended in every thread; the list was full): the direct
  // nibble sets staged over the properties windows, which no thread uses any more
  static_assert(region::kDirSets * region::kNibWords <= 256 * kPropsSlotWords, "dn fits the windows");
  __syncthreads();
  if ((lq_n[0] | lq_n[1] | lq_n[2] | lq_n[3]) == 0) return;
  uint32_t* dn = pwin;
  region::stage_direct_nib(dn, a.img);
  __syncthreads();
  const uint32_t nq = min(__builtin_amdgcn_readfirstlane(lq_n[wv]), kLongQ);
  for (uint32_t q = 0; q < nq; ++q) {
    const uint64_t pa = lq_jo[wv][q];
    const uint32_t c = region::record_crc_runs_wave(region::TabC{tbl}, nib, dn, g.base, rk, pa, lq_jl[wv][q], lane);
    if (lane == 0 && c != lq_ex[wv][q]) atomicOr(&a.status[lq_i[wv][q]], lq_bit[wv][q]);
  }
}

__global__ __launch_bounds__(256) void msg_reduce_kernel(MsgArgs a) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= a.m || (a.gate && *a.gate == 0)) return;
  uint32_t s = a.status[i];
#pragma unroll
  for (int k = 0; k < kMsgSlots; ++k) {
    const uint64_t j = (uint64_t)k * a.m + i;
    if (a.crc[j] != a.expected[j]) s |= record_bit(k);
  }
  a.status[i] = s;
}

// ---- CRC-trailered records: IndexSegment.checkDataIntegrityInByteBufferWithCRC
// (ambry-store/.../IndexSegment.java:727-735), the LogSegment header (LogSegment.java:130-140,
// 603-607), RestUtils user metadata (RestUtils.java:775-776, 813-814): the CRC of bytes
// [0, len - 8) compared, as a long, with the big-endian long in the last 8 bytes.
__global__ __launch_bounds__(256) void trailer_parse_kernel(TrailerArgs a) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= a.n) return;
  const uint64_t len = a.len[i];
  uint64_t jl = 0;
  uint32_t ex = 0;
  uint8_t force = 0;
  if (len < 8) {
    force = 1;  // the reference's limit(capacity - 8) throws: not intact
  } else {
    jl = len - 8;
    if (jl == 0 || jl > a.inline_max) {  // else the group phase reads it (SweepArgs::exp_fill)
      const uint64_t stored = be64(a.base + a.off[i] + jl);
      ex = (uint32_t)stored;
      force = (stored >> 32) ? 1 : 0;
    }
  }
  a.job_len[i] = jl;
  a.expected[i] = ex;
  a.force[i] = force;
}

__global__ __launch_bounds__(256) void trailer_verify_kernel(TrailerArgs a) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= a.n) return;
  const bool bad = a.force[i] || a.crc[i] != a.expected[i];
  if (a.mismatch) a.mismatch[i] = bad ? 1 : 0;
  if (bad && a.count) atomicAdd(a.count, 1u);
}

// ---------------------------------------------------------------- transform
// ValidatingTransformer.transform (ValidatingTransformer.java:46-104), after the verify pipeline
// set each message's status: one thread per message deserializes a clean PUT's fields the way
// deserializeBlobEncryptionKey / deserializeBlobProperties / deserializeUserMetadata /
// deserializeBlob read them (MessageFormatRecord.java:1568-1833) and describes the message
// PutMessageFormatInputStream would write from them (the fields stay in the region: the
// serializer copies them from there).
__device__ __forceinline__ bool gated_off(const uint32_t* gate, int when) {
  return gate && ((*gate != 0) != (when != 0));
}

// CRC of the V5 properties record from the stored record's CRC `c` (its bytes at rec, verified):
// the edits are XOR patterns at fixed places of an equal-length record, so each adds
// (crc(old window) ^ crc(new window)) * x^(8 * bytes after the window); the appended fields
// continue the CRC. No pass over the payload.
__device__ __forceinline__ uint32_t props_v5_crc(const uint32_t* __restrict__ img, const uint8_t* rec,
                                                 const PropsFix& x, uint32_t c) {
  if (!x.version) return c;
  const uint64_t L = 2ull + x.stored_len;  // record bytes the CRC covers
  uint8_t o[11], n[11];                    // record bytes [2, 13): SerDe version, ttl, private
#pragma unroll
  for (int k = 0; k < 11; ++k) o[k] = n[k] = rec[2 + k];
  n[0] = 0;
  n[1] = 5;
  n[kSerdePrivate] = x.priv;
  c ^= mul_xpow8_img(img, crc_bytes_img(img, 0u, o, 11) ^ crc_bytes_img(img, 0u, n, 11), L - 13);
  if (x.enc_pos) {
    const uint8_t eo = rec[2 + x.enc_pos], en = x.enc;
    if (eo != en)
      c ^= mul_xpow8_img(img, crc_bytes_img(img, 0u, &eo, 1) ^ crc_bytes_img(img, 0u, &en, 1),
                         L - (2ull + x.enc_pos + 1));
  }
  uint8_t app[kPropsAppendixMax];
  const uint32_t na = props_appendix(x.version, app);
  return crc_bytes_img(img, c, app, na);
}

// After the stored payloads are in place in the output: rewrite the re-encoded ones as V5.
__global__ __launch_bounds__(256) void props_fix_kernel(TransformArgs a) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= a.m || gated_off(a.gate, a.gate_when)) return;
  const ambrycrc_put_desc d = a.desc[i];
  if (d.header_version == 0) return;
  const PropsFix x = a.pfix[i];
  PutLayout L;
  if (!x.version || !put_layout(d, L)) return;
  props_apply_fix(a.out + d.out_off + (uint64_t)L.bp_rel + 2, x);
}

__device__ __forceinline__ void transform_describe(const TransformArgs& a, uint64_t i, uint32_t st0,
                                                   const PropsFields* pre) {
  uint32_t st = st0;
  ambrycrc_put_desc d;
  __builtin_memset(&d, 0, sizeof(d));  // header_version 0: nothing to write
  uint64_t out_len = 0;
  if (st == 0) {  // verified: the header and every record lie inside the region
    const uint64_t off = a.msg_off[i];
    const uint8_t* p = a.region + off;
    const uint32_t v = be16(p);
    const uint32_t hs = v == 1 ? 34u : v == 2 ? 38u : 40u;
    int32_t rel[5];
    int64_t total;
    uint32_t life = 0;
    if (v == 1) {
      total = (int64_t)be64(p + 2);
      rel[0] = -1;
      for (int k = 0; k < 4; ++k) rel[k + 1] = (int32_t)be32(p + 10 + 4 * k);
    } else if (v == 2) {
      total = (int64_t)be64(p + 2);
      for (int k = 0; k < 5; ++k) rel[k] = (int32_t)be32(p + 10 + 4 * k);
    } else {
      life = be16(p + 2);
      total = (int64_t)be64(p + 4);
      for (int k = 0; k < 5; ++k) rel[k] = (int32_t)be32(p + 12 + 4 * k);
    }
    const int32_t enc = rel[0], bp = rel[1], upd = rel[2], um = rel[3], blob = rel[4];
    if (upd != -1 || bp == -1 || um == -1 || blob == -1) {
      st |= AMBRYCRC_MSG_NOT_PUT;
    } else {
      const int64_t first = enc != -1 ? enc : bp;
      const int64_t end = first + total;  // message end, relative
      bool ok = first >= (int64_t)hs;
      uint32_t enc_len = 0;
      if (enc != -1) {  // BlobEncryptionKey_Format_V1: version, int size, key, CRC
        enc_len = be32(p + enc + 2);
        ok = ok && (int64_t)enc + 6 + enc_len + 8 == bp;
      }
      const int64_t props_len = (int64_t)um - bp - 2 - 8;  // BlobProperties_Format_V1: version, props, CRC
      const uint32_t um_len = be32(p + um + 2);             // UserMetadata_Format_V1: version, int size, ..., CRC
      ok = ok && props_len >= 0 && (int64_t)um + 6 + um_len + 8 == blob;
      // deserializeBlobProperties -> serializeBlobProperties at VERSION_5 (record_fields.h)
      PropsFields pf;
      if (pre) pf = *pre;  // the fused parse kernel parsed them already (from its LDS window)
      else ok = ok && props_parse<true>(p + bp + 2, (uint64_t)props_len, &pf) == 0;
      const bool encodable = !ok || pf.ascii;
      const PropsFix fx = ok ? props_fix_of(pf, (uint32_t)props_len) : PropsFix{};
      const uint32_t bv = be16(p + blob);  // Blob_Format_V1 / V2 / V3 (:1668-1833)
      uint32_t head = 0, type = 0, comp = 0;
      uint64_t size = 0;
      if (bv == 1) {
        size = be64(p + blob + 2);
        head = 10;
      } else if (bv == 2) {
        type = be16(p + blob + 2);
        size = be64(p + blob + 4);
        head = 12;
      } else if (bv == 3) {
        type = be16(p + blob + 2);
        comp = p[blob + 4] == 1 ? 1u : 0u;  // `readByte() == 1`
        size = be64(p + blob + 5);
        head = 13;
      } else {
        ok = false;
      }
      // BlobType has two values (DataBlob, MetadataBlob); sizes above Integer.MAX_VALUE throw
      ok = ok && type < 2 && size <= 0x7FFFFFFFull && (int64_t)blob + head + (int64_t)size + 8 == end;
      if (!ok) {
        st |= AMBRYCRC_MSG_BAD_RECORD;
      } else if (!encodable) {
        st |= AMBRYCRC_MSG_NOT_ENCODABLE;
      } else {
        d.key_src = off + hs;
        d.key_len = (uint32_t)(first - hs);
        const bool keep_enc = enc != -1 && a.header_version >= 2;
        d.enckey_src = keep_enc ? off + enc + 6 : 0;
        d.enckey_len = keep_enc ? (int32_t)enc_len : -1;
        d.props_src = off + bp + 2;
        d.props_len = props_v5_len(fx);
        a.pfix[i] = fx;
        d.usermeta_src = off + um + 6;
        d.usermeta_len = um_len;
        d.blob_src = off + blob + head;
        d.blob_len = size;
        d.life_version = a.life ? a.life[i] : (int16_t)life;
        d.blob_type = (int16_t)type;
        d.compressed = (uint8_t)comp;
        d.header_version = (uint8_t)a.header_version;
        PutLayout L;
        out_len = put_layout(d, L) ? L.length : 0;
        if (!out_len) {
          d.header_version = 0;
          st |= AMBRYCRC_MSG_BAD_RECORD;
        } else if (a.in_crc) {
          // every record of the input verified: its CRC is the low word of its 8-B trailer
          uint32_t* ic = a.in_crc + 4 * i;
          ic[0] = keep_enc ? be32(p + bp - 4) : 0u;
          ic[1] = props_v5_crc(a.img, p + bp, fx, be32(p + um - 4));
          ic[2] = be32(p + blob - 4);
          uint32_t cblob = be32(p + end - 4);
          if (bv != 3) {  // the V3 head (version 3, type, compressed, size) replaces a V1/V2 head
            // crc(B||C) = crc(A||C) ^ (crc(A) ^ crc(B)) * x^(8|C|)  (zlib's crc32_combine)
            uint8_t h3[13];
            put_be16(h3, 3u);
            put_be16(h3 + 2, type);
            h3[4] = (uint8_t)comp;
            put_be64(h3 + 5, size);
            const uint32_t ca = crc_bytes_img(a.img, 0u, p + blob, head);
            const uint32_t cb = crc_bytes_img(a.img, 0u, h3, 13);
            cblob ^= mul_xpow8_img(a.img, ca ^ cb, size);
          }
          ic[3] = cblob;
        }
      }
    }
  }
  a.desc[i] = d;
  a.out_len[i] = out_len;
  if (a.xstatus) a.xstatus[i] = st & ~st0;  // speculative: the transform's own bits, kept apart
  else a.status[i] = st;
}

__global__ __launch_bounds__(256) void transform_desc_kernel(TransformArgs a) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= a.m || gated_off(a.gate, a.gate_when)) return;
  transform_describe(a, i, a.status[i]);
}

// Packed placement: message i goes to start[i] (exclusive scan of out_len), if it fits.
__global__ __launch_bounds__(256) void transform_place_kernel(TransformArgs a, const uint64_t* __restrict__ start) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= a.m || gated_off(a.gate, a.gate_when)) return;
  const uint64_t len = a.out_len[i];
  uint64_t at = ~0ull;
  if (len) {
    if (start[i] + len <= a.out_cap) {
      at = start[i];
      a.desc[i].out_off = at;
    } else {
      a.desc[i].header_version = 0;
      a.out_len[i] = 0;
      if (a.xstatus) a.xstatus[i] |= AMBRYCRC_MSG_NO_ROOM;
      else a.status[i] |= AMBRYCRC_MSG_NO_ROOM;
    }
  }
  if (a.out_off) a.out_off[i] = at;
}

// Speculative pass: where the verify pass's copy-through puts each verify job (slot k of message
// i at k*m + i: encryption key, properties, update, user metadata, blob record) in the output.
// Records the output keeps byte for byte go to their output record start; the blob record goes
// so that its content lands at the output's content offset (a V1/V2 head, 10/12 B, lands inside
// the V3 head put_layout_kernel writes afterwards); the rest is read but not copied.
__global__ __launch_bounds__(256) void transform_jobs_kernel(TransformArgs a) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= a.m || gated_off(a.gate, a.gate_when)) return;
  const ambrycrc_put_desc d = a.desc[i];
  uint64_t co[kMsgSlots] = {kCopySkip, kCopySkip, kCopySkip, kCopySkip, kCopySkip};
  PutLayout L;
  if (d.header_version != 0 && put_layout(d, L)) {
    if (L.enc_rec) co[0] = d.out_off + (uint64_t)L.enc_rel;
    co[1] = d.out_off + (uint64_t)L.bp_rel;
    co[3] = d.out_off + (uint64_t)L.um_rel;
    const uint64_t in_head = d.blob_src - a.job_off[4 * a.m + i];  // both region offsets
    co[4] = d.out_off + (uint64_t)L.blob_rel + 13 - in_head;
  }
#pragma unroll
  for (int k = 0; k < kMsgSlots; ++k) a.copy_off[(uint64_t)k * a.m + i] = co[k];
}

// Speculative pass, after the verify: a placed message that failed verification sets `fail`
// (the fallback pass then rebuilds the output); a clean one gets its store key, the one field
// no verify job covers.
__global__ __launch_bounds__(256) void transform_finish_kernel(TransformArgs a) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= a.m || gated_off(a.gate, a.gate_when)) return;
  const ambrycrc_put_desc d = a.desc[i];
  if (d.header_version == 0) return;
  if (a.status[i] != 0) {
    atomicOr(a.fail, 1u);
    return;
  }
  const uint8_t* __restrict__ src = a.region + d.key_src;
  uint8_t* __restrict__ dst = a.out + d.out_off + (d.header_version == 1 ? 34u : d.header_version == 2 ? 38u : 40u);
  const uint32_t n = d.key_len;
  if (n < 8) {
    uint8_t t[8];
#pragma unroll
    for (uint32_t j = 0; j < 8; ++j) t[j] = j < n ? src[j] : 0;
#pragma unroll
    for (uint32_t j = 0; j < 8; ++j)
      if (j < n) dst[j] = t[j];
    return;
  }
  // 8-B moves at any alignment (unaligned global access), four loads in flight before their
  // stores; the last piece is [n - 8, n), overlapping the one before (one round trip per 32 B)
  for (uint32_t b0 = 0; b0 < n; b0 += 32) {
    uint64_t v[4];
#pragma unroll
    for (uint32_t u = 0; u < 4; ++u) __builtin_memcpy(&v[u], src + min(b0 + 8 * u, n - 8), 8);
#pragma unroll
    for (uint32_t u = 0; u < 4; ++u) __builtin_memcpy(dst + min(b0 + 8 * u, n - 8), &v[u], 8);
  }
}

// No fallback: the final status is the verify's bits, or else the transform's own.
__global__ __launch_bounds__(256) void transform_merge_kernel(TransformArgs a) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= a.m || gated_off(a.gate, a.gate_when) || (a.gate2 && *a.gate2 == 0)) return;
  if (a.status[i] == 0) a.status[i] = a.xstatus[i];
}

__global__ void xform_signal_kernel(const uint32_t* xfail, uint32_t* done, uint32_t seq) {
  if (threadIdx.x != 0) return;
  if (xfail && __hip_atomic_load(xfail, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0) return;
  __hip_atomic_store(done, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

hipError_t launch_xform_signal(const uint32_t* xfail, uint32_t* done, uint32_t seq, hipStream_t s) {
  hipLaunchKernelGGL(xform_signal_kernel, dim3(1), dim3(64), 0, s, xfail, done, seq);
  return hipGetLastError();
}

hipError_t launch_transform_jobs(const TransformArgs& a, hipStream_t s) {
  if (a.m == 0) return hipSuccess;
  hipLaunchKernelGGL(transform_jobs_kernel, dim3((uint32_t)((a.m + 255) / 256)), dim3(256), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_transform_finish(const TransformArgs& a, hipStream_t s) {
  if (a.m == 0) return hipSuccess;
  hipLaunchKernelGGL(transform_finish_kernel, dim3((uint32_t)((a.m + 255) / 256)), dim3(256), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_transform_merge(const TransformArgs& a, hipStream_t s) {
  if (a.m == 0) return hipSuccess;
  hipLaunchKernelGGL(transform_merge_kernel, dim3((uint32_t)((a.m + 255) / 256)), dim3(256), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_props_fix(const TransformArgs& a, hipStream_t s) {
  if (a.m == 0) return hipSuccess;
  hipLaunchKernelGGL(props_fix_kernel, dim3((uint32_t)((a.m + 255) / 256)), dim3(256), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_transform_desc(const TransformArgs& a, hipStream_t s) {
  if (a.m == 0) return hipSuccess;
  hipLaunchKernelGGL(transform_desc_kernel, dim3((uint32_t)((a.m + 255) / 256)), dim3(256), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_transform_place(const TransformArgs& a, const uint64_t* start, hipStream_t s) {
  if (a.m == 0) return hipSuccess;
  hipLaunchKernelGGL(transform_place_kernel, dim3((uint32_t)((a.m + 255) / 256)), dim3(256), 0, s, a, start);
  return hipGetLastError();
}

hipError_t launch_trailer_parse(const TrailerArgs& a, hipStream_t s) {
  if (a.n == 0) return hipSuccess;
  hipLaunchKernelGGL(trailer_parse_kernel, dim3((uint32_t)((a.n + 255) / 256)), dim3(256), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_trailer_verify(const TrailerArgs& a, hipStream_t s) {
  if (a.n == 0) return hipSuccess;
  hipLaunchKernelGGL(trailer_verify_kernel, dim3((uint32_t)((a.n + 255) / 256)), dim3(256), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_msg_parse(const MsgArgs& a, hipStream_t s) {
  if (a.m == 0) return hipSuccess;
  hipLaunchKernelGGL(msg_parse_kernel<false>, dim3(parse_blocks(a.m)), dim3(256), 0, s, a, TransformArgs{});
  return hipGetLastError();
}

hipError_t launch_msg_parse_desc(const MsgArgs& a, const TransformArgs& t, hipStream_t s) {
  if (a.m == 0) return hipSuccess;
  if (t.m != a.m || t.region != a.region || t.msg_off != a.msg_off) return hipErrorInvalidValue;
  hipLaunchKernelGGL(msg_parse_kernel<true>, dim3(parse_blocks(a.m)), dim3(256), 0, s, a, t);
  return hipGetLastError();
}

// Blocks per CU by message size (one box, ms per call, two interleaved runs; the
// kernel's 145 VGPRs allow 3 waves per SIMD): 2 blocks per CU 0.376 / 0.375 / 0.535 for 4 KiB /
// 1 KiB / 100-B blobs (5.3 / 2.2 / 1.3 KiB per message); 3: 0.383 / 0.391 / 0.522 -- more messages
// in flight pay only when each is small. Regions of at most kRegionSmallPerMessage bytes per
// message take AMBRY_REGION_BPC_SMALL blocks per CU.
constexpr uint64_t kRegionSmallPerMessage = 1536;
hipError_t launch_region_msg(const MsgArgs& a, const RegionArgs& g, int num_cu, hipStream_t s) {
  if (a.m == 0) return hipSuccess;
  const uint64_t bpc = a.region_len <= kRegionSmallPerMessage * a.m ? AMBRY_REGION_BPC_SMALL : AMBRY_REGION_BPC;
  uint64_t blocks = (a.m + 255) / 256;
  if (bpc > 0 && blocks > (uint64_t)num_cu * bpc) blocks = (uint64_t)num_cu * bpc;
  hipLaunchKernelGGL(region_msg_kernel, dim3((uint32_t)blocks), dim3(256), 0, s, a, g);
  return hipGetLastError();
}

// The long records the region kernels listed (LongList), piece by piece: wave w hashes pieces w,
// w + waves, ... (a static split; a claim loop through one atomic counter hung a two-pass verify on
// the GPU), each from the run sums (record_crc_runs_wave) into its slot, then counts it in the
// record's done word (release: fence, then the add); the wave that counts the last piece folds the
// record (acquire: fence after the add) -- no wave waits on another. Round 5's first form kept a
// per-record accumulator that 64 waves XORed into (28 us for eight 4 MiB blobs; then a second
// kernel folded each record in a 63-step Horner chain, 12.5 us).
__device__ __forceinline__ uint32_t long_count(const RegionArgs& g, uint32_t* total) {
  const unsigned long long ctr = __hip_atomic_load(g.lng.ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const uint32_t n = min((uint32_t)(ctr >> 32), g.lng.cap);
  *total = n ? min(g.lng.rec[n - 1].piece0 + g.lng.rec[n - 1].pieces, min((uint32_t)ctr, g.lng.pcap)) : 0u;
  return n;
}

// POW[k] = x^(8*2^k) nibble sets, k = 0..kLongPow-1, staged by region_long_kernel: the tree over
// 64 KiB pieces (k = 16..21), the fold over rounds of 64 pieces (22) and the last piece's length
// (0..16).
constexpr uint32_t kLongPow = 23;

// A record's CRC from its piece CRCs sl[0 .. np-1] (pieces 0 .. np-2 of kLongPiece bytes, the last
// of `last`), by the whole wave: the full pieces in rounds of 64 aligned so that piece np-2 is lane
// 63's, folded in-lane by x^(8*2^22) over the rounds, merged by the DPP tree (lane l takes lane
// l - 2^k's value times x^(8*2^(16+k))), then lane 63's register shifted by the last piece's length
// and the last piece's CRC added.
__device__ __forceinline__ uint32_t long_fold(const uint32_t* __restrict__ sl, uint32_t np, uint64_t last,
                                              const uint32_t* __restrict__ pw, uint32_t lane) {
  const uint32_t M = np - 1;  // full pieces
  uint32_t acc = 0;
  if (M) {
    const uint32_t V = (M + 63) / 64;
    for (uint32_t v = 0; v < V; ++v) {
      const int64_t j = (int64_t)64 * v + lane - ((int64_t)64 * V - M);
      const uint32_t x = j >= 0 ? sl[j] : 0u;
      acc = (v ? region::nmul(pw, acc, 22) : 0u) ^ x;
    }
    {
      const uint32_t pt = region::left_partner<0>(acc);
      if (lane & 1u) acc ^= region::nmul(pw, pt, 16);
    }
    {
      const uint32_t pt = region::left_partner<1>(acc);
      if (lane & 2u) acc ^= region::nmul(pw, pt, 17);
    }
    {
      const uint32_t pt = region::left_partner<2>(acc);
      if (lane & 4u) acc ^= region::nmul(pw, pt, 18);
    }
    {
      const uint32_t pt = region::left_partner<3>(acc);
      if (lane & 8u) acc ^= region::nmul(pw, pt, 19);
    }
    {
      const uint32_t pt = region::left_partner<4>(acc);
      if (lane & 16u) acc ^= region::nmul(pw, pt, 20);
    }
    {
      const uint32_t pt = region::left_partner<5>(acc);
      if (lane & 32u) acc ^= region::nmul(pw, pt, 21);
    }
    acc = (uint32_t)__builtin_amdgcn_readlane((int)acc, 63);
    for (uint32_t k = 0; k <= 16; ++k)  // acc x^(8 last), last = 1 .. kLongPiece (wave-uniform)
      if ((last >> k) & 1u) acc = region::nmul(pw, acc, k);
  }
  return acc ^ sl[np - 1];
}

__global__ __launch_bounds__(256) void region_long_kernel(MsgArgs a, RegionArgs g) {
  uint32_t total;
  const uint32_t n = long_count(g, &total);
  const uint32_t waves = gridDim.x * (blockDim.x >> 6);
  const uint32_t w0 = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  if (n == 0 || blockIdx.x * (blockDim.x >> 6) >= total) return;  // no piece for this block
  __shared__ uint32_t tbl[1024];
  __shared__ uint32_t nib[region::kNibTotal];
  __shared__ uint32_t dn[region::kDirSets * region::kNibWords];
  __shared__ uint32_t pw[kLongPow * region::kNibWords];
  stage_slice_tables(tbl, a.img);
  region::stage_nib(nib, a.img);
  region::stage_direct_nib(dn, a.img);
  for (uint32_t i = threadIdx.x; i < kLongPow * region::kNibWords; i += blockDim.x)
    pw[i] = a.img[(kNibBase + kPowOff) / 4 + i];  // POW[k] sets are consecutive, kNibWords apart
  __syncthreads();
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t* rk = g.rk + kRunPad;
  for (uint32_t q = w0; q < total; q += waves) {
    // the last record with piece0 <= q: 64 records a probe, one ballot each (one round trip for
    // up to 64 records)
    uint32_t lo = 0;
    for (uint32_t b = 0; b < n; b += 64) {
      const uint32_t r = b + lane;
      const uint64_t ball = __ballot(r < n && g.lng.rec[r].piece0 <= q);
      if (ball == 0) break;
      lo = b + 63u - (uint32_t)__builtin_clzll(ball);
      if (ball != ~0ull) break;
    }
    lo = __builtin_amdgcn_readfirstlane(lo);
    LongRec& lr = g.lng.rec[lo];
    const uint32_t p = q - lr.piece0, np = lr.pieces;
    if (p >= np) continue;  // a record listed empty
    const uint64_t s = (uint64_t)p * kLongPiece, e = min((uint64_t)lr.len, s + kLongPiece);
    const uint32_t c = region::record_crc_runs_wave(region::TabC{tbl}, nib, dn, g.base, rk, lr.pa + s, e - s, lane);
    if (lane == 0) g.lng.slot[q] = c;
    __threadfence();  // the slot before the count
    // Every lane runs the count (lane 0 adds 1, the rest 0: one atomic after the compiler's merge) so
    // the readfirstlane below follows no lane-0-only branch. A lane-0 atomic read back by readfirstlane
    // inside a loop is what hung round 5's claim loop: the compiler let lanes 1..63 re-enter the loop
    // without lane 0 and readfirstlane then read their own zero (DESIGN.md §11.3,
    // profiles/r06_hang_isa.txt; tests/test_kernel_lint.py forbids the pattern).
    const uint32_t prev = __builtin_amdgcn_readfirstlane(atomicAdd(&lr.done, lane == 0 ? 1u : 0u));
    if (prev + 1 != np) continue;
    __threadfence();  // every other piece's slot after its count
    const uint64_t last = (uint64_t)lr.len - (uint64_t)(np - 1) * kLongPiece;  // 1 .. kLongPiece
    const uint32_t crc = long_fold(g.lng.slot + lr.piece0, np, last, pw, lane);
    if (lane == 0 && crc != lr.ex) atomicOr(&a.status[lr.msg], lr.bit);
  }
}

hipError_t launch_region_long(const MsgArgs& a, const RegionArgs& g, int num_cu, hipStream_t s) {
  if (a.m == 0 || !g.lng.ctr) return hipSuccess;
  hipLaunchKernelGGL(region_long_kernel, dim3((uint32_t)num_cu * 2), dim3(256), 0, s, a, g);
  return hipGetLastError();
}

hipError_t launch_msg_reduce(const MsgArgs& a, hipStream_t s) {
  if (a.m == 0) return hipSuccess;
  hipLaunchKernelGGL(msg_reduce_kernel, dim3((uint32_t)((a.m + 255) / 256)), dim3(256), 0, s, a);
  return hipGetLastError();
}

}  // namespace ambrycrc
