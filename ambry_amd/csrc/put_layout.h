// put_layout.h -- byte layout of a PUT message (host and device), from
// PutMessageFormatInputStream.java:76-124 (header V2/V3, encryption-key record optional) and
// :133-162 (header V1), with the record formats of MessageFormatRecord.java:
//   header V1 (:467-486)  short 1, long totalSize, int bp, upd, um, blob relative offsets, CRC
//   header V2 (:696-725)  short 2, long totalSize, int enc, bp, upd, um, blob, CRC
//   header V3 (:951-981)  short 3, short lifeVersion, long totalSize, int enc, bp, upd, um, blob, CRC
//   BlobEncryptionKey_Format_V1 (:1568-1601)  short 1, int size, key, CRC
//   BlobProperties_Format_V1 (:1162-1195)     short 1, BlobPropertiesSerDe bytes, CRC
//   UserMetadata_Format_V1 (:1619-1650)       short 1, int size, metadata, CRC
//   Blob_Format_V3 (:1777-1833)               short 3, short blobType, byte isCompressed, long size,
//                                             content, CRC
// totalSize counts the records after the key; the update-record offset is always -1 for a PUT.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/ambrycrc.h"

namespace ambrycrc {

constexpr uint32_t kPutSlots = 5;  // CRC jobs per message: header, encryption key, properties, user metadata, blob

struct PutLayout {
  uint32_t hsize;     // header bytes
  uint64_t enc_rec;   // record sizes (enc_rec 0 when absent)
  uint64_t props_rec;
  uint64_t um_rec;
  uint64_t blob_rec;
  uint64_t total;     // header totalSize
  int32_t enc_rel;    // relative offsets from the message start (-1 when absent)
  int32_t bp_rel;
  int32_t um_rel;
  int32_t blob_rel;   // fits in an int for the header; checked by put_layout_ok
  uint64_t length;    // whole message
};

__host__ __device__ inline bool put_layout(const ambrycrc_put_desc& d, PutLayout& L) {
  const int v = d.header_version;
  if (v < 1 || v > 3) return false;
  if (d.enckey_len < -1 || (v == 1 && d.enckey_len >= 0)) return false;
  L.hsize = v == 1 ? 34u : v == 2 ? 38u : 40u;
  L.enc_rec = d.enckey_len >= 0 ? 2ull + 4 + (uint64_t)d.enckey_len + 8 : 0;
  L.props_rec = 2ull + d.props_len + 8;
  L.um_rec = 2ull + 4 + d.usermeta_len + 8;
  L.blob_rec = 13ull + d.blob_len + 8;
  L.total = L.enc_rec + L.props_rec + L.um_rec + L.blob_rec;
  const uint64_t key_end = (uint64_t)L.hsize + d.key_len;
  const uint64_t bp = key_end + L.enc_rec, um = bp + L.props_rec, blob = um + L.um_rec;
  if (blob > 0x7FFFFFFFull) return false;  // relative offsets are Java ints
  L.enc_rel = d.enckey_len >= 0 ? (int32_t)key_end : -1;
  L.bp_rel = (int32_t)bp;
  L.um_rel = (int32_t)um;
  L.blob_rel = (int32_t)blob;
  L.length = blob + L.blob_rec;
  return true;
}

// Big-endian stores at any alignment (one unaligned store each on the device and the host).
__host__ __device__ inline void put_be16(uint8_t* p, uint32_t v) {
  const uint16_t x = __builtin_bswap16((uint16_t)v);
  __builtin_memcpy(p, &x, 2);
}
__host__ __device__ inline void put_be32(uint8_t* p, uint32_t v) {
  const uint32_t x = __builtin_bswap32(v);
  __builtin_memcpy(p, &x, 4);
}
__host__ __device__ inline void put_be64(uint8_t* p, uint64_t v) {
  const uint64_t x = __builtin_bswap64(v);
  __builtin_memcpy(p, &x, 8);
}

// The header's CRC'd bytes [0, hsize - 8) (26, 30 or 32) into h; returns their count.
__host__ __device__ inline uint32_t put_header_bytes(const ambrycrc_put_desc& d, const PutLayout& L, uint8_t (&h)[32]) {
  const int v = d.header_version;
  h[30] = h[31] = 0;
  put_be16(h, (uint32_t)v);
  if (v == 3) {
    put_be16(h + 2, (uint32_t)(uint16_t)d.life_version);
    put_be64(h + 4, L.total);
    put_be32(h + 12, (uint32_t)L.enc_rel);
    put_be32(h + 16, (uint32_t)L.bp_rel);
    put_be32(h + 20, 0xFFFFFFFFu);  // update record: Message_Header_Invalid_Relative_Offset
    put_be32(h + 24, (uint32_t)L.um_rel);
    put_be32(h + 28, (uint32_t)L.blob_rel);
    return 32;
  }
  put_be64(h + 2, L.total);
  if (v == 2) {
    put_be32(h + 10, (uint32_t)L.enc_rel);
    put_be32(h + 14, (uint32_t)L.bp_rel);
    put_be32(h + 18, 0xFFFFFFFFu);
    put_be32(h + 22, (uint32_t)L.um_rel);
    put_be32(h + 26, (uint32_t)L.blob_rel);
    return 30;
  }
  put_be32(h + 10, (uint32_t)L.bp_rel);
  put_be32(h + 14, 0xFFFFFFFFu);
  put_be32(h + 18, (uint32_t)L.um_rel);
  put_be32(h + 22, (uint32_t)L.blob_rel);
  return 26;
}

// Record k's prefix (k = 1 encryption key, 2 properties, 3 user metadata, 4 blob): the bytes
// before its variable field that its CRC covers -- version, and the size (key, metadata) or
// type, isCompressed and size (blob) fields. Into b; returns the count (6, 2, 6, 13).
__host__ __device__ inline uint32_t put_prefix_bytes(const ambrycrc_put_desc& d, uint32_t k, uint8_t (&b)[16]) {
  switch (k) {
    case 1:
      put_be16(b, 1);
      put_be32(b + 2, (uint32_t)d.enckey_len);
      return 6;
    case 2:
      put_be16(b, 1);
      return 2;
    case 3:
      put_be16(b, 1);
      put_be32(b + 2, d.usermeta_len);
      return 6;
    default:
      put_be16(b, 3);
      put_be16(b + 2, (uint32_t)(uint16_t)d.blob_type);
      b[4] = d.compressed ? 1 : 0;
      put_be64(b + 5, d.blob_len);
      return 13;
  }
}

// Record k's offset from the message start (k as put_prefix_bytes).
__host__ __device__ inline int32_t put_record_rel(const PutLayout& L, uint32_t k) {
  return k == 1 ? L.enc_rel : k == 2 ? L.bp_rel : k == 3 ? L.um_rel : L.blob_rel;
}

// Header (without its CRC) and the fixed prefixes of every record, at message start m
// (constant-size copies: on the device one wide unaligned store per 16 B, not a store per byte).
__host__ __device__ inline void put_write_fixed(const ambrycrc_put_desc& d, const PutLayout& L, uint8_t* m) {
  uint8_t h[32];
  const uint32_t n = put_header_bytes(d, L, h);
  if (n == 32) __builtin_memcpy(m, h, 32);
  else if (n == 30) __builtin_memcpy(m, h, 30);
  else __builtin_memcpy(m, h, 26);
  uint8_t b[16];
  if (L.enc_rec) {
    put_prefix_bytes(d, 1, b);
    __builtin_memcpy(m + L.enc_rel, b, 6);
  }
  put_prefix_bytes(d, 2, b);
  __builtin_memcpy(m + L.bp_rel, b, 2);
  put_prefix_bytes(d, 3, b);
  __builtin_memcpy(m + L.um_rel, b, 6);
  put_prefix_bytes(d, 4, b);
  __builtin_memcpy(m + L.blob_rel, b, 13);
}

// Offsets (from the message start) of the variable fields: key, encryption key, properties,
// user metadata, blob content.
__host__ __device__ inline void put_field_offsets(const ambrycrc_put_desc& d, const PutLayout& L, uint64_t* o) {
  o[0] = L.hsize;
  o[1] = L.enc_rec ? (uint64_t)L.enc_rel + 6 : 0;
  o[2] = (uint64_t)L.bp_rel + 2;
  o[3] = (uint64_t)L.um_rel + 6;
  o[4] = (uint64_t)L.blob_rel + 13;
  (void)d;
}

// CRC job k of the message: [off, off + len) relative to its start; the trailer follows at off + len.
__host__ __device__ inline void put_crc_job(const PutLayout& L, uint32_t k, uint64_t* off, uint64_t* len,
                                            bool* present) {
  *present = true;
  switch (k) {
    case 0: *off = 0; *len = L.hsize - 8; break;
    case 1:
      *present = L.enc_rec != 0;
      *off = L.enc_rec ? (uint64_t)L.enc_rel : 0;
      *len = L.enc_rec ? L.enc_rec - 8 : 0;
      break;
    case 2: *off = (uint64_t)L.bp_rel; *len = L.props_rec - 8; break;
    case 3: *off = (uint64_t)L.um_rel; *len = L.um_rec - 8; break;
    default: *off = (uint64_t)L.blob_rel; *len = L.blob_rec - 8; break;
  }
}

}  // namespace ambrycrc
