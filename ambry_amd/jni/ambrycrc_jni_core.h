/*
 * ambrycrc_jni_core.h -- the JNI shim's argument checking and marshalling, as plain C with no
 * JNI types (built into libambrycrc_jnicore.so, tested through ctypes in tests/test_jni_core.py;
 * ambrycrc_jni.c only moves Java values in and out and throws what these functions report).
 *
 * Every check the reference's Java makes before touching bytes is made here again in C, so a
 * bad offset from any caller raises instead of reading out of bounds:
 *   java.util.zip.CRC32.update(byte[],off,len): off < 0, len < 0 or off + len > length
 *     -> ArrayIndexOutOfBoundsException (the behaviour CrcInputStream/CrcOutputStream rely on,
 *     CrcInputStream.java:58-62, CrcOutputStream.java:48-57)
 *   Crc32.update(ByteBuffer) reads position..limit of the buffer (Crc32.java:100-143)
 */
#ifndef AMBRYCRC_JNI_CORE_H
#define AMBRYCRC_JNI_CORE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* What the JNI layer throws for a status (AJC_* below or AMBRYCRC_E*). */
#define AJC_OK 0
#define AJC_EBOUNDS (-100)    /* offset/length outside the array or buffer -> IndexOutOfBoundsException */
#define AJC_ENOTDIRECT (-101) /* a ByteBuffer without a native address -> IllegalArgumentException */
#define AJC_ESHORT (-102)     /* an output/parameter array shorter than the batch -> IllegalArgumentException */
#define AJC_ENULL (-103)      /* a required array or buffer is null -> NullPointerException */

/* Java class name (JNI form) of the exception for `status`, or NULL for AJC_OK. Negative
 * AMBRYCRC_E* codes map to java/lang/IllegalStateException (ENOMEM: java/lang/OutOfMemoryError). */
const char* ajc_exception_class(int status);
/* Exception message for `status` (static string). */
const char* ajc_message(int status);

/* 1 iff 0 <= off, 0 <= len and off + len <= cap (no overflow), else 0. */
int ajc_range_ok(int64_t cap, int64_t off, int64_t len);

/* *out = the CRC continued over base[off, off+len) of an array/buffer of cap bytes; the CRC slot
 * is never used for a status. base may be NULL only when len == 0. */
int ajc_update(uint32_t crc, const uint8_t* base, int64_t cap, int64_t off, int64_t len, uint32_t* out);

/* Batch over n direct buffers (NativeCrc32.batch): buffer i is bases[i] with capacity caps[i]
 * (NULL base: not direct), chunk [pos[i], pos[i] + len[i]). Fills ptrs/lens for
 * ambrycrc_batch_host; on error *bad = the first offending index. */
int ajc_batch_args(size_t n, const uint8_t* const* bases, const int64_t* caps, const int32_t* pos,
                   const int32_t* len, const void** ptrs, uint64_t* lens, size_t* bad);

/* Gather list (NativeCrc32.updateAll): buffer i's bytes are [pos[i], lim[i]); pos <= lim <= cap. */
int ajc_iov_args(size_t n, const uint8_t* const* bases, const int64_t* caps, const int32_t* pos,
                 const int32_t* lim, const void** ptrs, size_t* lens, size_t* bad);

/* Array lengths of a batch call: every parameter array holds at least n entries (a length of -1
 * stands for an optional array passed as null). */
int ajc_batch_lengths(int64_t n, int64_t pos_len, int64_t len_len, int64_t crc_in_len, int64_t out_len);

/* nativeVerifyMessages: m offsets; status holds >= m entries; ends (-1: null) too. */
int ajc_verify_lengths(int64_t m, int64_t status_len, int64_t ends_len);

/* nativeTransformMessages: m offsets; status, outLens, outOffsets (-1: null) and lifeVersions (-1: null)
 * hold >= m entries each. */
int ajc_transform_lengths(int64_t m, int64_t life_len, int64_t out_off_len, int64_t out_len_len, int64_t status_len);

/* nativePutCrcs: n = blobCrc.length; blobLen holds >= n; wireOut and its fields list (-1 each: null), recordOut
 * and its prefixes list likewise hold >= n entries. An output without its input list is AJC_ENULL. */
int ajc_put_lengths(int64_t n, int64_t blob_len_len, int64_t fields_len, int64_t wire_len, int64_t prefixes_len,
                    int64_t record_len);

/* nativeRangeChecksums: n = first.length; second and out hold >= n entries. */
int ajc_range_lengths(int64_t n, int64_t second_len, int64_t out_len);

#ifdef __cplusplus
}
#endif
#endif
