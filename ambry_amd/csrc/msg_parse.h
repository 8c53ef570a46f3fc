// msg_parse.h -- one stored message's header, record checks and CRC jobs, for the thread-per-
// message kernels of the message verify and transform (message_kernels.hip) and the region-mode
// message processors (crc32_kernels.hip region_fused_kernel / region_tail_kernel).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/ambrycrc.h"
#include "crc32_kernels.h"
#include "record_fields.h"

namespace ambrycrc {

// Big-endian fields at arbitrary byte offsets: one unaligned global load each (gfx9 global
// memory runs in unaligned access mode; the compiler emits global_load_dword[x2] for these
// memcpys), where byte-wise reads cost a load per byte.
__device__ __forceinline__ uint32_t be16(const uint8_t* p) {
  uint16_t v;
  __builtin_memcpy(&v, p, 2);
  return __builtin_bswap16(v);
}
__device__ __forceinline__ uint32_t be32(const uint8_t* p) {
  uint32_t v;
  __builtin_memcpy(&v, p, 4);
  return __builtin_bswap32(v);
}
__device__ __forceinline__ uint64_t be64(const uint8_t* p) {
  uint64_t v;
  __builtin_memcpy(&v, p, 8);
  return __builtin_bswap64(v);
}

// The status bit of record slot k (encryption key, properties, update, user metadata, blob).
static_assert(AMBRYCRC_MSG_ENCKEY_CRC == 2u && AMBRYCRC_MSG_PROPS_CRC == 4u && AMBRYCRC_MSG_UPDATE_CRC == 8u &&
                  AMBRYCRC_MSG_USERMETA_CRC == 16u && AMBRYCRC_MSG_BLOB_CRC == 32u,
              "record bits are consecutive");
__device__ __forceinline__ uint32_t record_bit(int k) { return AMBRYCRC_MSG_ENCKEY_CRC << k; }

// Header bytes [0, 40) of a message as ten little-endian words, one unaligned 16 + 16 + 8 B
// load when the region holds 40 bytes past `off` (the longest header, V3), else byte loads
// with zero fill. Issued before the table staging, so one memory round trip covers it.
struct HeaderWords {
  uint32_t w[10];
};

__device__ __forceinline__ HeaderWords load_header(const uint8_t* p, uint64_t rem) {
  HeaderWords h;
  if (rem >= 40) {
    __builtin_memcpy(&h.w[0], p, 16);
    __builtin_memcpy(&h.w[4], p + 16, 16);
    __builtin_memcpy(&h.w[8], p + 32, 8);
  } else {
#pragma unroll
    for (int i = 0; i < 10; ++i) {
      uint32_t v = 0;
#pragma unroll
      for (int b = 0; b < 4; ++b)
        if ((uint64_t)(4 * i + b) < rem) v |= (uint32_t)p[4 * i + b] << (8 * b);
      h.w[i] = v;
    }
  }
  return h;
}

// Big-endian 32-bit field at byte 4k+2 (V1/V2 layouts) and at byte 4k (V3) of the header.
__device__ __forceinline__ uint32_t be32_w2(const HeaderWords& h, int k) {
  return __builtin_bswap32(__builtin_amdgcn_alignbyte(h.w[k + 1], h.w[k], 2));
}
__device__ __forceinline__ uint32_t be32_w0(const HeaderWords& h, int k) { return __builtin_bswap32(h.w[k]); }

// CRC-32 of the first n = h - 8 header bytes (26, 30 or 32) from the words: slice-by-4 over
// whole words, then the two trailing bytes of V1/V2.
__device__ __forceinline__ uint32_t header_crc(const HeaderWords& h, uint32_t n, const uint32_t* __restrict__ t) {
  uint32_t c = 0xFFFFFFFFu;
  const uint32_t nw = n >> 2;
#pragma unroll
  for (uint32_t i = 0; i < 8; ++i) {
    if (i < nw) {
      const uint32_t x = c ^ h.w[i];
      c = t[768 + (x & 0xffu)] ^ t[512 + ((x >> 8) & 0xffu)] ^ t[256 + ((x >> 16) & 0xffu)] ^ t[x >> 24];
    }
  }
  if (n & 2u) {
    const uint32_t tw = nw == 6 ? h.w[6] : h.w[7];
    c = (c >> 8) ^ t[(c ^ tw) & 0xffu];
    c = (c >> 8) ^ t[(c ^ (tw >> 8)) & 0xffu];
  }
  return ~c;
}

// What each record's deserializer reads before its CRC (MessageFormatRecord.java), for a record
// of `span` bytes at q (its stored CRC the last 8): the record version (an unknown one throws
// UnknownFormatVersion, :147-239) and the size fields that decide where the stream looks for
// the CRC. BlobEncryptionKey_Format_V1 (:1588-1600) and UserMetadata_Format_V1 (:1637-1649): an
// int size, then that many bytes, then the CRC; Blob_Format_V1/V2/V3 (:1681-1833): blob type
// ordinal < 2, a long size <= Integer.MAX_VALUE, then the content and the CRC. A size that
// disagrees with the header's record span, or a bad type, is AMBRYCRC_MSG_BAD_RECORD (the
// reference reads the CRC at a different place, or throws). BlobProperties_Format_V1 and
// Update_Format_V1..V3: their fields, to the CRC (record_fields.h).
__device__ __forceinline__ uint32_t record_check(int k, const uint8_t* q, uint64_t span) {
  if (span < 10) return AMBRYCRC_MSG_BAD_RECORD;  // a version and a CRC at least
  const uint32_t v = be16(q);
  switch (k) {
    case 0:    // encryption key
    case 3: {  // user metadata
      if (v != 1) return AMBRYCRC_MSG_BAD_VERSION;
      if (span < 14) return AMBRYCRC_MSG_BAD_RECORD;
      const int32_t n = (int32_t)be32(q + 2);
      return n >= 0 && (uint64_t)n + 14 == span ? 0u : AMBRYCRC_MSG_BAD_RECORD;
    }
    case 1:  // properties (msg_parse_kernel parses them from its LDS window instead)
      return props_record_check(q, span);
    case 2:  // update
      return update_record_check(q, span);
    default: {  // blob
      if (v < 1 || v > 3) return AMBRYCRC_MSG_BAD_VERSION;
      const uint32_t head = v == 1 ? 10u : v == 2 ? 12u : 13u;
      if (span < head + 8) return AMBRYCRC_MSG_BAD_RECORD;
      const uint32_t type = v == 1 ? 0u : be16(q + 2);
      const uint64_t size = be64(q + (v == 1 ? 2 : v == 2 ? 4 : 5));
      return type < 2 && size <= 0x7FFFFFFFull && size + head + 8 == span ? 0u : AMBRYCRC_MSG_BAD_RECORD;
    }
  }
}


// The first bytes of a record staged in this thread's LDS slot, the rest read from global memory:
// the properties parse walks int-length strings, one dependent read per field, which from LDS
// costs an LDS round trip instead of a memory one.
constexpr uint32_t kPropsWin = AMBRY_PROPS_WIN;        // bytes staged per thread (a multiple of 16)
constexpr uint32_t kPropsSlotWords = kPropsWin / 4 + 1;  // +1 word: consecutive slots start on consecutive banks
struct WinBytes {
  const uint8_t* w;  // LDS copy of [0, n)
  const uint8_t* g;  // the same bytes in global memory
  uint32_t n;
  __device__ uint32_t u8(uint64_t i) const { return i < n ? w[i] : g[i]; }
  __device__ uint32_t be16(uint64_t i) const { return i + 2 <= n ? (uint32_t)w[i] << 8 | w[i + 1] : ld_be16(g + i); }
  __device__ uint32_t be32(uint64_t i) const {
    return i + 4 <= n ? (uint32_t)w[i] << 24 | (uint32_t)w[i + 1] << 16 | (uint32_t)w[i + 2] << 8 | w[i + 3]
                      : ld_be32(g + i);
  }
  __device__ bool ascii(uint64_t i, uint64_t len) const {
    if (i + len > n) return bytes_ascii(g + i, len);
    uint32_t acc = 0;
    for (uint64_t j = 0; j < len; ++j) acc |= w[i + j];
    return acc < 0x80u;
  }
};

// One message's header, record checks and CRC jobs (job k = [jo[k], jo[k] + jl[k]) from the
// region start, its stored CRC ex[k]; records of 1..inline_max bytes leave ex[k] to the group
// phase). slot: this thread's LDS window for the properties. DESC: the transform's ASCII scan.
struct MsgParse {
  uint64_t jo[kMsgSlots] = {0, 0, 0, 0, 0}, jl[kMsgSlots] = {0, 0, 0, 0, 0};
  uint32_t ex[kMsgSlots] = {0, 0, 0, 0, 0};
  uint32_t status = 0;
  uint64_t end = 0;
};

// WIN = false: no LDS window; the properties are parsed from memory (the region-mode processors,
// whose region bytes were just streamed past and sit in the caches).
template <bool DESC, bool WIN = true>
__device__ __forceinline__ void parse_message(uint64_t off, bool in_region, uint64_t rem, const uint8_t* p,
                                              const HeaderWords& hw, const uint32_t* __restrict__ tbl,
                                              uint32_t* __restrict__ slot, uint64_t inline_max, MsgParse& r,
                                              PropsFields& pf, bool& pf_ok) {
  do {
    if (!in_region || rem < 2) {
      r.status = AMBRYCRC_MSG_BAD_LAYOUT;
      break;
    }
    const int v = (int16_t)__builtin_bswap16((uint16_t)hw.w[0]);
    const uint32_t h = v == 1 ? 34u : v == 2 ? 38u : v == 3 ? 40u : 0u;
    if (h == 0) {
      r.status = AMBRYCRC_MSG_BAD_VERSION;
      break;
    }
    if (rem < h) {
      r.status = AMBRYCRC_MSG_BAD_LAYOUT;
      break;
    }
    // stored header CRC: bytes [h-8, h)
    const uint32_t st_hi = v == 3 ? be32_w0(hw, 8) : v == 2 ? be32_w2(hw, 7) : be32_w2(hw, 6);
    const uint32_t st_lo = v == 3 ? be32_w0(hw, 9) : v == 2 ? be32_w2(hw, 8) : be32_w2(hw, 7);
    if (st_hi != 0 || header_crc(hw, h - 8, tbl) != st_lo) {  // verifyHeader: nothing else is read
      r.status = AMBRYCRC_MSG_HEADER_CRC;
      break;
    }
    int64_t total;
    int32_t rel[kMsgSlots];
    if (v == 3) {
      if ((int16_t)__builtin_bswap16((uint16_t)(hw.w[0] >> 16)) < 0) {  // lifeVersion >= 0
        r.status = AMBRYCRC_MSG_BAD_LAYOUT;
        break;
      }
      total = (int64_t)(((uint64_t)be32_w0(hw, 1) << 32) | be32_w0(hw, 2));
#pragma unroll
      for (int k = 0; k < 5; ++k) rel[k] = (int32_t)be32_w0(hw, 3 + k);
    } else {
      total = (int64_t)(((uint64_t)be32_w2(hw, 0) << 32) | be32_w2(hw, 1));
      if (v == 1) {
        rel[0] = -1;
#pragma unroll
        for (int k = 0; k < 4; ++k) rel[k + 1] = (int32_t)be32_w2(hw, 2 + k);
      } else {
#pragma unroll
        for (int k = 0; k < 5; ++k) rel[k] = (int32_t)be32_w2(hw, 2 + k);
      }
    }
    // checkHeaderConstraints (MessageFormatRecord.java:985-1030), exact put / update shapes
    const bool is_put = rel[1] != -1 && rel[2] == -1 && rel[3] != -1 && rel[4] != -1;
    const bool is_upd = rel[2] != -1 && rel[0] == -1 && rel[1] == -1 && rel[3] == -1 && rel[4] == -1;
    if (total <= 0 || !(is_put || is_upd)) {
      r.status = AMBRYCRC_MSG_BAD_LAYOUT;
      break;
    }
    int64_t prev = -1, first = -1;
    bool ok = true;
    for (int k = 0; k < kMsgSlots; ++k) {
      if (rel[k] == -1) continue;
      if (rel[k] <= prev || rel[k] < (int32_t)h) ok = false;
      if (first < 0) first = rel[k];
      prev = rel[k];
    }
    if (!ok || (uint64_t)total > rem || (uint64_t)first > rem - (uint64_t)total) {
      r.status = AMBRYCRC_MSG_BAD_LAYOUT;
      break;
    }
    r.end = (uint64_t)first + (uint64_t)total;
    uint64_t rend[kMsgSlots];  // end of record k (its stored CRC's last byte + 1)
    for (int k = 0; k < kMsgSlots; ++k) {
      rend[k] = r.end;
      for (int j = k + 1; j < kMsgSlots; ++j)
        if (rel[j] != -1) {
          rend[k] = (uint64_t)rel[j];
          break;
        }
      if (rel[k] != -1 && rend[k] < (uint64_t)rel[k] + 8) ok = false;
    }
    if (!ok) {
      r.status = AMBRYCRC_MSG_BAD_LAYOUT;
      r.end = 0;
      break;
    }
    if (!WIN && rel[1] != -1) {  // properties parsed from memory
      const uint8_t* q = p + rel[1];
      const uint64_t span = rend[1] - (uint64_t)rel[1];
      uint32_t ps = AMBRYCRC_MSG_BAD_RECORD;
      if (span >= 10) ps = be16(q) != 1 ? AMBRYCRC_MSG_BAD_VERSION : props_parse_b<DESC>(MemBytes{q + 2}, span - 10, &pf);
      pf_ok = ps == 0;
      r.status |= ps;
    }
    if (WIN && rel[1] != -1) {  // properties: staged, then parsed (the transform's ASCII scan too: DESC)
      const uint8_t* q = p + rel[1];
      const uint64_t avail = rem - (uint64_t)rel[1];
      const uint32_t w = (uint32_t)(avail < kPropsWin ? avail : kPropsWin) & ~15u;
      uint32_t v[kPropsWin / 4];
#pragma unroll
      for (uint32_t j = 0; j < kPropsWin / 16; ++j)
        if (16 * j + 16 <= w) __builtin_memcpy(&v[4 * j], q + 16 * j, 16);  // one round trip
#pragma unroll
      for (uint32_t j = 0; j < kPropsWin / 4; ++j)
        if (4 * j + 4 <= w) slot[j] = v[j];
      const uint64_t span = rend[1] - (uint64_t)rel[1];
      uint32_t ps = AMBRYCRC_MSG_BAD_RECORD;
      if (span >= 10) {
        const uint32_t ver = w >= 2 ? (uint32_t)reinterpret_cast<const uint8_t*>(slot)[0] << 8 |
                                          reinterpret_cast<const uint8_t*>(slot)[1]
                                    : be16(q);
        ps = ver != 1 ? AMBRYCRC_MSG_BAD_VERSION
                      : props_parse_b<DESC>(WinBytes{reinterpret_cast<const uint8_t*>(slot) + 2, q + 2,
                                                     w >= 2 ? w - 2 : 0u},
                                            span - 10, &pf);
      }
      pf_ok = ps == 0;
      r.status |= ps;
    }
    for (int k = 0; k < kMsgSlots; ++k) {
      if (rel[k] == -1) continue;
      const uint64_t e = rend[k];
      if (k != 1) r.status |= record_check(k, p + rel[k], e - (uint64_t)rel[k]);
      r.jo[k] = off + (uint64_t)rel[k];
      r.jl[k] = e - (uint64_t)rel[k] - 8;
      // Records the group phase takes whole have their stored CRC read there, from the line
      // it is already streaming (SweepArgs::exp_fill); only the others cost a fetch here.
      if (r.jl[k] == 0 || r.jl[k] > inline_max) {
        const uint64_t stored = be64(p + e - 8);
        if (stored >> 32) r.status |= record_bit(k);  // a CRC32 never has upper bits: mismatch regardless
        r.ex[k] = (uint32_t)stored;
      }
    }
  } while (false);
}

// The end of the message the header describes (first record + total size), or 0 when the header
// is unparseable or the message overruns `rem` -- what parse_message would read up to, from the
// header words alone (no CRC check): the region-mode processors' wait target.
__device__ __forceinline__ uint64_t header_end(const HeaderWords& hw, uint64_t rem) {
  if (rem < 2) return 0;
  const int v = (int16_t)__builtin_bswap16((uint16_t)hw.w[0]);
  const uint32_t h = v == 1 ? 34u : v == 2 ? 38u : v == 3 ? 40u : 0u;
  if (h == 0 || rem < h) return 0;
  int64_t total;
  int32_t first = -1;
  if (v == 3) {
    total = (int64_t)(((uint64_t)be32_w0(hw, 1) << 32) | be32_w0(hw, 2));
    for (int k = 4; k >= 0; --k)
      if ((int32_t)be32_w0(hw, 3 + k) != -1) first = (int32_t)be32_w0(hw, 3 + k);
  } else {
    total = (int64_t)(((uint64_t)be32_w2(hw, 0) << 32) | be32_w2(hw, 1));
    const int nk = v == 1 ? 4 : 5;
    for (int k = nk - 1; k >= 0; --k)
      if ((int32_t)be32_w2(hw, 2 + k) != -1) first = (int32_t)be32_w2(hw, 2 + k);
  }
  if (total <= 0 || first < 0 || (uint64_t)total > rem || (uint64_t)first > rem - (uint64_t)total) return 0;
  return (uint64_t)first + (uint64_t)total;
}

}  // namespace ambrycrc
