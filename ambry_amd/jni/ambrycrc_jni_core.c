/* ambrycrc_jni_core.c -- see ambrycrc_jni_core.h. Plain C, no JNI types. */
#include "ambrycrc_jni_core.h"

#include "../../include/ambrycrc.h"

const char* ajc_exception_class(int status) {
  switch (status) {
    case AJC_OK: return NULL;
    case AJC_EBOUNDS: return "java/lang/IndexOutOfBoundsException";
    case AJC_ENOTDIRECT:
    case AJC_ESHORT:
    case AMBRYCRC_EINVAL: return "java/lang/IllegalArgumentException";
    case AJC_ENULL: return "java/lang/NullPointerException";
    case AMBRYCRC_ENOMEM: return "java/lang/OutOfMemoryError";
    default: return "java/lang/IllegalStateException";
  }
}

const char* ajc_message(int status) {
  switch (status) {
    case AJC_OK: return "ok";
    case AJC_EBOUNDS: return "offset/length outside the array or buffer";
    case AJC_ENOTDIRECT: return "ByteBuffer is not direct (no native address)";
    case AJC_ESHORT: return "parameter array shorter than the batch";
    case AJC_ENULL: return "null array or buffer";
    default: return ambrycrc_strerror(status);
  }
}

int ajc_range_ok(int64_t cap, int64_t off, int64_t len) {
  return cap >= 0 && off >= 0 && len >= 0 && off <= cap && len <= cap - off;
}

int ajc_update(uint32_t crc, const uint8_t* base, int64_t cap, int64_t off, int64_t len, uint32_t* out) {
  if (!out) return AMBRYCRC_EINVAL;
  if (!ajc_range_ok(cap, off, len)) return AJC_EBOUNDS;
  if (len == 0) {
    *out = crc;
    return AJC_OK;
  }
  if (!base) return AJC_ENULL;
  *out = ambrycrc_update(crc, base + off, (size_t)len);
  return AJC_OK;
}

int ajc_batch_args(size_t n, const uint8_t* const* bases, const int64_t* caps, const int32_t* pos,
                   const int32_t* len, const void** ptrs, uint64_t* lens, size_t* bad) {
  if (n && (!bases || !caps || !pos || !len || !ptrs || !lens)) return AJC_ENULL;
  for (size_t i = 0; i < n; ++i) {
    if (bad) *bad = i;
    if (!bases[i]) return AJC_ENOTDIRECT;
    if (!ajc_range_ok(caps[i], pos[i], len[i])) return AJC_EBOUNDS;
    ptrs[i] = bases[i] + pos[i];
    lens[i] = (uint64_t)len[i];
  }
  return AJC_OK;
}

int ajc_iov_args(size_t n, const uint8_t* const* bases, const int64_t* caps, const int32_t* pos,
                 const int32_t* lim, const void** ptrs, size_t* lens, size_t* bad) {
  if (n && (!bases || !caps || !pos || !lim || !ptrs || !lens)) return AJC_ENULL;
  for (size_t i = 0; i < n; ++i) {
    if (bad) *bad = i;
    if (!bases[i]) return AJC_ENOTDIRECT;
    if (pos[i] < 0 || lim[i] < pos[i] || !ajc_range_ok(caps[i], pos[i], (int64_t)lim[i] - pos[i])) return AJC_EBOUNDS;
    ptrs[i] = bases[i] + pos[i];
    lens[i] = (size_t)(lim[i] - pos[i]);
  }
  return AJC_OK;
}

int ajc_batch_lengths(int64_t n, int64_t pos_len, int64_t len_len, int64_t crc_in_len, int64_t out_len) {
  if (n < 0 || pos_len < 0 || len_len < 0 || out_len < 0) return AJC_ENULL;
  if (pos_len < n || len_len < n || out_len < n || (crc_in_len >= 0 && crc_in_len < n)) return AJC_ESHORT;
  return AJC_OK;
}

int ajc_verify_lengths(int64_t m, int64_t status_len, int64_t ends_len) {
  if (m < 0 || status_len < 0) return AJC_ENULL;
  if (status_len < m || (ends_len >= 0 && ends_len < m)) return AJC_ESHORT;
  return AJC_OK;
}

int ajc_transform_lengths(int64_t m, int64_t life_len, int64_t out_off_len, int64_t out_len_len, int64_t status_len) {
  if (m < 0 || out_len_len < 0 || status_len < 0) return AJC_ENULL;
  if (status_len < m || out_len_len < m || (out_off_len >= 0 && out_off_len < m) || (life_len >= 0 && life_len < m))
    return AJC_ESHORT;
  return AJC_OK;
}

int ajc_put_lengths(int64_t n, int64_t blob_len_len, int64_t fields_len, int64_t wire_len, int64_t prefixes_len,
                    int64_t record_len) {
  if (n < 0 || blob_len_len < 0) return AJC_ENULL;
  if ((wire_len >= 0 && fields_len < 0) || (record_len >= 0 && prefixes_len < 0)) return AJC_ENULL;
  if (blob_len_len < n) return AJC_ESHORT;
  if (wire_len >= 0 && (wire_len < n || fields_len < n)) return AJC_ESHORT;
  if (record_len >= 0 && (record_len < n || prefixes_len < n)) return AJC_ESHORT;
  return AJC_OK;
}

int ajc_range_lengths(int64_t n, int64_t second_len, int64_t out_len) {
  if (n < 0 || second_len < 0 || out_len < 0) return AJC_ENULL;
  if (second_len < n || out_len < n) return AJC_ESHORT;
  return AJC_OK;
}
