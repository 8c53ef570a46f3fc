// record_fields.h -- the field reads of the two variable-layout records, shared by the device
// verify / transform (message_kernels.hip) and the per-message CPU path (ambrycrc_msg_cpu.cpp):
//
//   BlobProperties_Format_V1 payload = BlobPropertiesSerDe bytes (BlobPropertiesSerDe.java:56-77):
//     short version (1..5), long ttl, byte private, long creationTime, long blobSize,
//     int-string contentType, ownerId, serviceId,
//     [v > 1] short accountId, short containerId,  [v > 2] byte encrypted,
//     [v > 3] nullable int-string contentEncoding, filename,  [v > 4] reservedMetadataBlobId
//   Update_Format_V1..V3 (MessageFormatRecord.java:1200-1480)
//
// Every function reads only inside the span it is given: a field past it is the EOFException.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/ambrycrc.h"

namespace ambrycrc {

__host__ __device__ inline uint32_t ld_be16(const uint8_t* p) {
  uint16_t v;
  __builtin_memcpy(&v, p, 2);
  return __builtin_bswap16(v);
}
__host__ __device__ inline uint32_t ld_be32(const uint8_t* p) {
  uint32_t v;
  __builtin_memcpy(&v, p, 4);
  return __builtin_bswap32(v);
}

constexpr uint32_t kSerdeFixed = 27;  // version, ttl, private, creationTime, blobSize
constexpr uint32_t kSerdePrivate = 10;  // offset of the `private` byte

struct PropsFields {
  uint32_t version;   // 1..5
  uint32_t enc_pos;   // offset of the `encrypted` byte (version >= 3), else 0
  uint8_t priv_raw;   // the stored bytes
  uint8_t enc_raw;    // 0 below version 3
  bool ascii;         // every string byte < 0x80 (computed only when asked)
};

// Whether n bytes at p are all < 0x80: 8-B unaligned loads, OR-reduced.
__host__ __device__ inline bool bytes_ascii(const uint8_t* p, uint64_t n) {
  uint64_t acc = 0;
  uint64_t i = 0;
  for (; i + 8 <= n; i += 8) {
    uint64_t w;
    __builtin_memcpy(&w, p + i, 8);
    acc |= w;
  }
  for (; i < n; ++i) acc |= p[i];
  return (acc & 0x8080808080808080ull) == 0;
}

// Byte source of a parse: plain memory (host, or device global memory).
struct MemBytes {
  const uint8_t* p;
  __host__ __device__ uint32_t u8(uint64_t i) const { return p[i]; }
  __host__ __device__ uint32_t be16(uint64_t i) const { return ld_be16(p + i); }
  __host__ __device__ uint32_t be32(uint64_t i) const { return ld_be32(p + i); }
  __host__ __device__ bool ascii(uint64_t i, uint64_t n) const { return bytes_ascii(p + i, n); }
};

// BlobPropertiesSerDe.getBlobPropertiesFromStream over the n bytes at s (the record's payload:
// its span minus the 2-B record version and the 8-B CRC). 0, or AMBRYCRC_MSG_BAD_RECORD when a
// read throws (unknown SerDe version, a negative string size, a field past the span --
// BlobProperties_Format_V1.deserializeBlobPropertiesRecord maps each to DataCorrupt,
// MessageFormatRecord.java:1192-1195) or the fields end before the span does (the reference would
// take other bytes for the CRC). ASCII: also scan the string bytes (the transform's question).
template <bool ASCII, class B>
__host__ __device__ inline uint32_t props_parse_b(const B& s, uint64_t n, PropsFields* f) {
  if (n < kSerdeFixed) return AMBRYCRC_MSG_BAD_RECORD;
  const int32_t v = (int16_t)s.be16(0);
  if (v < 1 || v > 5) return AMBRYCRC_MSG_BAD_RECORD;  // "stream has unknown blob property version"
  f->version = (uint32_t)v;
  f->priv_raw = (uint8_t)s.u8(kSerdePrivate);
  f->enc_raw = 0;
  f->enc_pos = 0;
  bool ascii = true;
  uint64_t pos = kSerdeFixed;
  // three readIntString, then (v > 3) two readNullableIntString, then (v > 4) one more;
  // the account/container shorts and the encrypted byte sit after the first three
  const uint32_t nstr = v > 4 ? 6u : v > 3 ? 5u : 3u;
  for (uint32_t k = 0; k < nstr; ++k) {
    if (k == 3) {
      pos += v > 1 ? 4u : 0u;
      if (v > 2) {
        if (pos + 1 > n) return AMBRYCRC_MSG_BAD_RECORD;
        f->enc_pos = (uint32_t)pos;
        f->enc_raw = (uint8_t)s.u8(pos);
        pos += 1;
      }
    }
    if (pos + 4 > n) return AMBRYCRC_MSG_BAD_RECORD;
    const int32_t len = (int32_t)s.be32(pos);
    pos += 4;
    if (len < 0 || (uint64_t)len > n - pos) return AMBRYCRC_MSG_BAD_RECORD;
    if (ASCII) ascii = ascii && s.ascii(pos, (uint64_t)len);
    pos += (uint64_t)len;
  }
  if (nstr == 3) {  // V1..V3: the shorts / byte follow the last string
    pos += v > 1 ? 4u : 0u;
    if (v > 2) {
      if (pos + 1 > n) return AMBRYCRC_MSG_BAD_RECORD;
      f->enc_pos = (uint32_t)pos;
      f->enc_raw = (uint8_t)s.u8(pos);
      pos += 1;
    }
    if (pos > n) return AMBRYCRC_MSG_BAD_RECORD;
  }
  f->ascii = ascii;
  return pos == n ? 0u : AMBRYCRC_MSG_BAD_RECORD;
}

template <bool ASCII>
__host__ __device__ inline uint32_t props_parse(const uint8_t* s, uint64_t n, PropsFields* f) {
  return props_parse_b<ASCII>(MemBytes{s}, n, f);
}

// The BlobProperties record check of verify: record version 1 (else UnknownFormatVersion,
// MessageFormatRecord.java:143-155), then the SerDe fields over [q + 2, q + span - 8).
__host__ __device__ inline uint32_t props_record_check(const uint8_t* q, uint64_t span) {
  if (ld_be16(q) != 1) return AMBRYCRC_MSG_BAD_VERSION;
  PropsFields f;
  return props_parse<false>(q + 2, span - 10, &f);
}

// deserializeUpdateRecord (MessageFormatRecord.java:158-172) for a record of `span` bytes (stored
// CRC included, span >= 10): V1 (:1217-1228) a byte; V2 (:1253-1266) account, container, update
// time; V3 (:1388-1413) those, a short type indexing SubRecord.Type.values() {DELETE, TTL_UPDATE,
// UNDELETE} (out of range throws), the sub-record's short version (1, else UnknownFormatVersion,
// :1422-1464) and for TTL_UPDATE a long expiry. The fields must end at the CRC.
__host__ __device__ inline uint32_t update_record_check(const uint8_t* q, uint64_t span) {
  const uint32_t v = ld_be16(q);
  const uint64_t body = span - 8;
  if (v == 1) return body == 3 ? 0u : AMBRYCRC_MSG_BAD_RECORD;
  if (v == 2) return body == 14 ? 0u : AMBRYCRC_MSG_BAD_RECORD;
  if (v != 3) return AMBRYCRC_MSG_BAD_VERSION;
  if (body < 16) return AMBRYCRC_MSG_BAD_RECORD;
  const int32_t type = (int16_t)ld_be16(q + 14);
  if (type < 0 || type > 2) return AMBRYCRC_MSG_BAD_RECORD;
  if (body < 18) return AMBRYCRC_MSG_BAD_RECORD;
  if (ld_be16(q + 16) != 1) return AMBRYCRC_MSG_BAD_VERSION;
  return body == (type == 1 ? 26u : 18u) ? 0u : AMBRYCRC_MSG_BAD_RECORD;
}

// ---- the transform's V5 re-encoding (BlobPropertiesSerDe.serializeBlobProperties at
// CURRENT_VERSION = VERSION_5, BlobPropertiesSerDe.java:41,83-103, of what props_parse read).
// With every string ASCII the output is the stored bytes with
//   [0, 2) = 5, [10] = private == 1, [enc_pos] = encrypted == 1 (version >= 3)
// and the fields older versions lack appended (they all come after the stored bytes):
//   V1: account -1, container -1 (Account/Container.UNKNOWN_*_ID), encrypted 0, three int 0 (null
//   strings); V2: encrypted 0 + three int 0; V3: three int 0; V4: one int 0 (reserved); V5: none.
// A non-ASCII string byte is AMBRYCRC_MSG_NOT_ENCODABLE: the reference re-encodes each string
// (decoded as UTF-8) with the default charset, so it outgrows the String.length() budget of
// getBlobPropertiesSerDeSize (:43-54, Utils.getIntStringLength, Utils.java:233-235) and overruns
// PutMessageFormatInputStream's buffer (PutMessageFormatInputStream.java:83-90): the transform
// throws (ValidatingTransformer.java:100-102). UTF-8 default charset assumed.
constexpr uint32_t kPropsAppendixMax = 17;

__host__ __device__ inline uint32_t props_appendix(uint32_t version, uint8_t (&a)[kPropsAppendixMax]) {
  const uint32_t n = version == 1 ? 17u : version == 2 ? 13u : version == 3 ? 12u : version == 4 ? 4u : 0u;
  for (uint32_t i = 0; i < kPropsAppendixMax; ++i) a[i] = 0;
  if (version == 1) a[0] = a[1] = a[2] = a[3] = 0xFF;
  return n;
}

// What the transform must change in a stored payload of stored_len bytes to make its V5 bytes
// (16 B, per message, in the transform's workspace). version 0: nothing (already canonical V5).
struct PropsFix {
  uint32_t stored_len;
  uint32_t enc_pos;   // 0: no encrypted byte to rewrite
  uint8_t version;    // stored SerDe version, 0 = no change
  uint8_t priv;       // canonical bytes
  uint8_t enc;
  uint8_t pad[5];
};
static_assert(sizeof(PropsFix) == 16, "PropsFix");

__host__ __device__ inline PropsFix props_fix_of(const PropsFields& f, uint32_t stored_len) {
  PropsFix x;
  x.stored_len = stored_len;
  x.priv = f.priv_raw == 1 ? 1 : 0;
  x.enc = f.enc_raw == 1 ? 1 : 0;
  x.enc_pos = f.version >= 3 ? f.enc_pos : 0u;
  const bool canonical = f.version == 5 && x.priv == f.priv_raw && x.enc == f.enc_raw;
  x.version = canonical ? 0 : (uint8_t)f.version;
  for (int i = 0; i < 5; ++i) x.pad[i] = 0;
  return x;
}

__host__ __device__ inline uint32_t props_v5_len(const PropsFix& x) {
  uint8_t a[kPropsAppendixMax];
  return x.stored_len + (x.version ? props_appendix(x.version, a) : 0u);
}

// Rewrite the stored payload at s (stored_len bytes already there) into its V5 bytes in place.
__host__ __device__ inline void props_apply_fix(uint8_t* s, const PropsFix& x) {
  if (!x.version) return;
  s[0] = 0;
  s[1] = 5;
  s[kSerdePrivate] = x.priv;
  if (x.enc_pos) s[x.enc_pos] = x.enc;
  uint8_t a[kPropsAppendixMax];
  const uint32_t n = props_appendix(x.version, a);
  for (uint32_t i = 0; i < n; ++i) s[x.stored_len + i] = a[i];
}

}  // namespace ambrycrc
