/*
 * ambrycrc_jni.c -- JNI shim binding com.github.ambry.utils.NativeCrc32
 * (integration/java/com/github/ambry/utils/NativeCrc32.java) to libambrycrc's C ABI
 * (include/ambrycrc.h).
 *
 * Built for a JVM where a JDK provides jni.h (`make -C ambry_amd jni JAVA_HOME=...`). This build
 * image has no JDK: tests/test_jni_core.py compiles this file against a test-only
 * JNI subset (tests/native/jni_stub/jni.h) and runs it in a fake JVM (tests/native/jni_harness.c).
 * Its argument checks and marshalling live in ambrycrc_jni_core.c (plain C, tested through
 * ctypes); this file only moves Java values in and out.
 *
 * Errors never travel in the CRC slot: a failed check or a native error throws (the matching
 * java.lang exception from ajc_exception_class) and the native method returns; the Java
 * caller sees the pending exception. Every offset and length is checked against the array
 * length or the direct buffer's capacity here, whatever the Java wrapper already checked.
 *
 * Java natives served:
 *   int  nativeUpdateArray(int crc, byte[] b, int off, int len)       Crc32.java:55-98
 *   int  nativeUpdateDirect(int crc, ByteBuffer buf, int pos, int len) Crc32.java:100-143
 *   int  nativeUpdateByte(int crc, int b)                              Crc32.java:146-148
 *   int  nativeUpdateDirectAll(int crc, ByteBuffer[] bufs)             PutOperation.java:2041-2043
 *   int  nativeCombine(int crc1, int crc2, long len2)
 *   void nativeInit(int device)
 *   void nativeBatchDirect(ByteBuffer[] bufs, int[] pos, int[] len, int[] crcIn, int[] out, int device)
 *   void nativeVerifyMessages(ByteBuffer region, long[] offsets, int[] status, long[] ends, int device)
 *   int  nativeVerifyMessage(ByteBuffer region, long offset, long[] end)
 *   int  nativeChainMessages(ByteBuffer region, long start, long[] offsets)
 *   int  nativeTransformMessage(ByteBuffer region, long offset, int lifeVersion, int headerVersion,
 *                               ByteBuffer out, long[] outLen)
 *   void nativeTransformMessages(ByteBuffer region, long[] offsets, short[] lifeVersions, int headerVersion,
 *                                ByteBuffer out, long[] outOffsets, long[] outLens, int[] status, int device)
 *   void nativePutCrcs(ByteBuffer[] fields, ByteBuffer[] prefixes, int[] blobCrc, long[] blobLen,
 *                      int[] wireOut, int[] recordOut)                  PutRequest.java:238-283
 *   void nativeRangeChecksums(ByteBuffer file, long[] first, long[] second, int[] out, int device)
 *                                                                      FileStore.java:567-595
 *   int  nativeSetHostPolicy(int device, int policy)
 *   int  nativeSetHostCpuThreads(int device, int threads)
 *   int  nativeHostRates(int device, double[] out)
 *   int  nativeLastHostPath(int device)
 * CRC values travel as Java ints holding the uint32 bit pattern.
 */
#include <jni.h>
#include <stdint.h>
#include <stdlib.h>

#include "../../include/ambrycrc.h"
#include "ambrycrc_jni_core.h"

#define JNI_FN(name) Java_com_github_ambry_utils_NativeCrc32_##name

/* Throws the exception for `status` (no-op for AJC_OK, or when one is already pending). */
static int raise(JNIEnv* env, int status) {
  if (status == AJC_OK) return 0;
  if ((*env)->ExceptionCheck(env)) return 1;
  jclass cls = (*env)->FindClass(env, ajc_exception_class(status));
  if (cls) (*env)->ThrowNew(env, cls, ajc_message(status));
  return 1;
}

/* Direct buffer address and capacity (NULL / -1 when the buffer is not direct). */
static const uint8_t* direct(JNIEnv* env, jobject buf, int64_t* cap) {
  *cap = -1;
  if (!buf) return NULL;
  const uint8_t* p = (const uint8_t*)(*env)->GetDirectBufferAddress(env, buf);
  if (p) *cap = (int64_t)(*env)->GetDirectBufferCapacity(env, buf);
  return p;
}

JNIEXPORT void JNICALL JNI_FN(nativeInit)(JNIEnv* env, jclass cls, jint device) {
  (void)cls;
  raise(env, ambrycrc_init(device));
}

/* Crc32.update(byte[] b, int off, int len) -- Crc32.java:55-98. The array is pinned with
 * GetPrimitiveArrayCritical only for the host-side update. */
JNIEXPORT jint JNICALL JNI_FN(nativeUpdateArray)(JNIEnv* env, jclass cls, jint crc, jbyteArray b, jint off,
                                                 jint len) {
  (void)cls;
  if (!b) return raise(env, AJC_ENULL), crc;
  const int64_t cap = (*env)->GetArrayLength(env, b);
  if (!ajc_range_ok(cap, off, len)) return raise(env, AJC_EBOUNDS), crc;
  if (len == 0) return crc;
  jbyte* p = (jbyte*)(*env)->GetPrimitiveArrayCritical(env, b, NULL);
  if (!p) return raise(env, AMBRYCRC_ENOMEM), crc;  /* the JVM usually has an OOM pending already */
  uint32_t r = 0;
  const int st = ajc_update((uint32_t)crc, (const uint8_t*)p, cap, off, len, &r);
  (*env)->ReleasePrimitiveArrayCritical(env, b, p, JNI_ABORT);
  if (raise(env, st)) return crc;
  return (jint)r;
}

/* Crc32.update(ByteBuffer) on a direct buffer (Crc32.java:100-143); the Java side then sets
 * position(limit) as the reference method does. */
JNIEXPORT jint JNICALL JNI_FN(nativeUpdateDirect)(JNIEnv* env, jclass cls, jint crc, jobject buf, jint pos,
                                                  jint len) {
  (void)cls;
  int64_t cap;
  const uint8_t* p = direct(env, buf, &cap);
  if (!buf) return raise(env, AJC_ENULL), crc;
  if (!p) return raise(env, AJC_ENOTDIRECT), crc;
  uint32_t r = 0;
  if (raise(env, ajc_update((uint32_t)crc, p, cap, pos, len, &r))) return crc;
  return (jint)r;
}

/* Crc32.update(int b) -- Crc32.java:146-148. */
JNIEXPORT jint JNICALL JNI_FN(nativeUpdateByte)(JNIEnv* env, jclass cls, jint crc, jint b) {
  (void)env;
  (void)cls;
  return (jint)ambrycrc_update_byte((uint32_t)crc, b);
}

JNIEXPORT jint JNICALL JNI_FN(nativeCombine)(JNIEnv* env, jclass cls, jint crc1, jint crc2, jlong len2) {
  (void)cls;
  if (len2 < 0) return raise(env, AMBRYCRC_EINVAL), 0;
  return (jint)ambrycrc_combine((uint32_t)crc1, (uint32_t)crc2, (uint64_t)len2);
}

/* Batch of direct ByteBuffers (Netty nioBuffers / registered arenas) -> device path
 * (ambrycrc_batch_host: pinned staging, hipMemcpyAsync, gfx950 kernels). */
JNIEXPORT void JNICALL JNI_FN(nativeBatchDirect)(JNIEnv* env, jclass cls, jobjectArray bufs, jintArray pos,
                                                 jintArray len, jintArray crc_in, jintArray out, jint device) {
  (void)cls;
  if (!bufs || !pos || !len || !out) {
    raise(env, AJC_ENULL);
    return;
  }
  const jsize n = (*env)->GetArrayLength(env, bufs);
  if (raise(env, ajc_batch_lengths(n, (*env)->GetArrayLength(env, pos), (*env)->GetArrayLength(env, len),
                                   crc_in ? (*env)->GetArrayLength(env, crc_in) : -1,
                                   (*env)->GetArrayLength(env, out))))
    return;
  if (n == 0) return;
  const uint8_t** bases = (const uint8_t**)malloc(sizeof(void*) * (size_t)n);
  int64_t* caps = (int64_t*)malloc(sizeof(int64_t) * (size_t)n);
  jint* jpos = (jint*)malloc(sizeof(jint) * (size_t)n);
  jint* jlen = (jint*)malloc(sizeof(jint) * (size_t)n);
  const void** ptrs = (const void**)malloc(sizeof(void*) * (size_t)n);
  uint64_t* lens = (uint64_t*)malloc(sizeof(uint64_t) * (size_t)n);
  uint32_t* cin = crc_in ? (uint32_t*)malloc(sizeof(uint32_t) * (size_t)n) : NULL;
  uint32_t* res = (uint32_t*)malloc(sizeof(uint32_t) * (size_t)n);
  int st = AMBRYCRC_ENOMEM;
  if (bases && caps && jpos && jlen && ptrs && lens && res && (!crc_in || cin)) {
    (*env)->GetIntArrayRegion(env, pos, 0, n, jpos);
    (*env)->GetIntArrayRegion(env, len, 0, n, jlen);
    if (crc_in) (*env)->GetIntArrayRegion(env, crc_in, 0, n, (jint*)cin);
    for (jsize i = 0; i < n; ++i) {
      jobject b = (*env)->GetObjectArrayElement(env, bufs, i);
      bases[i] = direct(env, b, &caps[i]);
      (*env)->DeleteLocalRef(env, b);
    }
    size_t bad = 0;
    st = ajc_batch_args((size_t)n, bases, caps, jpos, jlen, ptrs, lens, &bad);
    if (st == AJC_OK) st = ambrycrc_batch_host(ptrs, lens, cin, res, (size_t)n, device, 0);
    if (st == AJC_OK) (*env)->SetIntArrayRegion(env, out, 0, n, (const jint*)res);
  }
  free(bases);
  free(caps);
  free(jpos);
  free(jlen);
  free(ptrs);
  free(lens);
  free(cin);
  free(res);
  raise(env, st);
}

/* Verify every CRC of the PUT / update messages at `offsets` in a direct ByteBuffer holding a
 * log-segment region (BlobStoreRecovery.java:43-110 scan, MessageFormatSend.java:131-139 on
 * GET, ValidatingTransformer.java:46-104 on replication) -> ambrycrc_verify_messages_host.
 * status[i]: AMBRYCRC_MSG_* bits (0 = every CRC matches); ends[i]: message end or 0. Offsets
 * past the region are data (BAD_LAYOUT), not an error. */
JNIEXPORT void JNICALL JNI_FN(nativeVerifyMessages)(JNIEnv* env, jclass cls, jobject region, jlongArray offsets,
                                                    jintArray status, jlongArray ends, jint device) {
  (void)cls;
  if (!region || !offsets || !status) {
    raise(env, AJC_ENULL);
    return;
  }
  const jsize m = (*env)->GetArrayLength(env, offsets);
  if (raise(env, ajc_verify_lengths(m, (*env)->GetArrayLength(env, status),
                                    ends ? (*env)->GetArrayLength(env, ends) : -1)))
    return;
  int64_t cap;
  const uint8_t* base = direct(env, region, &cap);
  if (!base) {
    raise(env, AJC_ENOTDIRECT);
    return;
  }
  if (m == 0) return;
  uint64_t* offs = (uint64_t*)malloc(sizeof(uint64_t) * (size_t)m);
  uint32_t* st = (uint32_t*)malloc(sizeof(uint32_t) * (size_t)m);
  uint64_t* en = ends ? (uint64_t*)malloc(sizeof(uint64_t) * (size_t)m) : NULL;
  int rc = AMBRYCRC_ENOMEM;
  if (offs && st && (!ends || en)) {
    (*env)->GetLongArrayRegion(env, offsets, 0, m, (jlong*)offs); /* jlong and uint64_t: same width */
    rc = ambrycrc_verify_messages_host(base, (uint64_t)cap, offs, (size_t)m, st, en, device, 0);
    if (rc == AMBRYCRC_OK) {
      (*env)->SetIntArrayRegion(env, status, 0, m, (const jint*)st);
      if (ends) (*env)->SetLongArrayRegion(env, ends, 0, m, (const jlong*)en);
    }
  }
  free(offs);
  free(st);
  free(en);
  raise(env, rc);
}

/* position..limit of buffers[0 .. n) (each non-null and direct) into ptrs / lens; a status. */
static int gather_list(JNIEnv* env, jobjectArray bufs, jsize n, const void** ptrs, size_t* lens) {
  if (n == 0) return AJC_OK;
  jclass bc = (*env)->FindClass(env, "java/nio/Buffer");
  jmethodID mpos = bc ? (*env)->GetMethodID(env, bc, "position", "()I") : NULL;
  jmethodID mlim = bc ? (*env)->GetMethodID(env, bc, "limit", "()I") : NULL;
  if (!mpos || !mlim) return AMBRYCRC_EINVAL;
  const uint8_t** bases = (const uint8_t**)malloc(sizeof(void*) * (size_t)n);
  int64_t* caps = (int64_t*)malloc(sizeof(int64_t) * (size_t)n);
  jint* jpos = (jint*)malloc(sizeof(jint) * (size_t)n);
  jint* jlim = (jint*)malloc(sizeof(jint) * (size_t)n);
  int st = AMBRYCRC_ENOMEM;
  if (bases && caps && jpos && jlim) {
    st = AJC_OK;
    for (jsize i = 0; i < n && st == AJC_OK; ++i) {
      jobject b = (*env)->GetObjectArrayElement(env, bufs, i);
      if (!b) {
        st = AJC_ENULL;
        break;
      }
      bases[i] = direct(env, b, &caps[i]);
      jpos[i] = (*env)->CallIntMethod(env, b, mpos);
      jlim[i] = (*env)->CallIntMethod(env, b, mlim);
      (*env)->DeleteLocalRef(env, b);
      if ((*env)->ExceptionCheck(env)) st = AMBRYCRC_EINVAL;
    }
    size_t bad = 0;
    if (st == AJC_OK) st = ajc_iov_args((size_t)n, bases, caps, jpos, jlim, ptrs, lens, &bad);
  }
  free(bases);
  free(caps);
  free(jpos);
  free(jlim);
  return st;
}

/* The loop of PutOperation.PutChunk.verifyCRC (PutOperation.java:2041-2043) over a Netty
 * CompositeByteBuf's nioBuffers(), all direct: one JNI crossing for the whole gather list
 * (ambrycrc_update_iov). Each buffer's position..limit is used; the Java side consumes them. */
JNIEXPORT jint JNICALL JNI_FN(nativeUpdateDirectAll)(JNIEnv* env, jclass cls, jint crc, jobjectArray bufs) {
  (void)cls;
  if (!bufs) return raise(env, AJC_ENULL), crc;
  const jsize n = (*env)->GetArrayLength(env, bufs);
  if (n == 0) return crc;
  const void** ptrs = (const void**)malloc(sizeof(void*) * (size_t)n);
  size_t* lens = (size_t*)malloc(sizeof(size_t) * (size_t)n);
  jint result = crc;
  int st = AMBRYCRC_ENOMEM;
  if (ptrs && lens) {
    st = gather_list(env, bufs, n, ptrs, lens);
    if (st == AJC_OK) result = (jint)ambrycrc_update_iov((uint32_t)crc, ptrs, lens, (size_t)n);
  }
  free(ptrs);
  free(lens);
  raise(env, st);
  return result;
}

/* NativeCrc32.putCrcs -> ambrycrc_put_crcs: PutRequest.prepareBuffer's wire CRC
 * (PutRequest.java:238-283) and the Blob_Format_V3 record CRC (MessageFormatRecord.java:1789-1795,
 * PutMessageFormatInputStream.java:116-120) of n PUTs from their known blob CRCs, by GF(2) combine.
 * fields[i] / prefixes[i]: direct buffers, position..limit used (not consumed). */
JNIEXPORT void JNICALL JNI_FN(nativePutCrcs)(JNIEnv* env, jclass cls, jobjectArray fields, jobjectArray prefixes,
                                             jintArray blob_crc, jlongArray blob_len, jintArray wire_out,
                                             jintArray record_out) {
  (void)cls;
  if (!blob_crc || !blob_len) {
    raise(env, AJC_ENULL);
    return;
  }
  const jsize n = (*env)->GetArrayLength(env, blob_crc);
  if (raise(env, ajc_put_lengths(n, (*env)->GetArrayLength(env, blob_len),
                                 fields ? (*env)->GetArrayLength(env, fields) : -1,
                                 wire_out ? (*env)->GetArrayLength(env, wire_out) : -1,
                                 prefixes ? (*env)->GetArrayLength(env, prefixes) : -1,
                                 record_out ? (*env)->GetArrayLength(env, record_out) : -1)))
    return;
  if (n == 0 || (!wire_out && !record_out)) return;
  uint32_t* crc = (uint32_t*)malloc(sizeof(uint32_t) * (size_t)n);
  uint64_t* blen = (uint64_t*)malloc(sizeof(uint64_t) * (size_t)n);
  const void** fp = (const void**)malloc(sizeof(void*) * (size_t)n);
  size_t* fl = (size_t*)malloc(sizeof(size_t) * (size_t)n);
  const void** pp = (const void**)malloc(sizeof(void*) * (size_t)n);
  size_t* pl = (size_t*)malloc(sizeof(size_t) * (size_t)n);
  uint64_t* fl64 = (uint64_t*)malloc(sizeof(uint64_t) * (size_t)n);
  uint64_t* pl64 = (uint64_t*)malloc(sizeof(uint64_t) * (size_t)n);
  uint32_t* wire = (uint32_t*)malloc(sizeof(uint32_t) * (size_t)n);
  uint32_t* rec = (uint32_t*)malloc(sizeof(uint32_t) * (size_t)n);
  int st = AMBRYCRC_ENOMEM;
  if (crc && blen && fp && fl && pp && pl && fl64 && pl64 && wire && rec) {
    (*env)->GetIntArrayRegion(env, blob_crc, 0, n, (jint*)crc);
    (*env)->GetLongArrayRegion(env, blob_len, 0, n, (jlong*)blen);
    st = AJC_OK;
    for (jsize i = 0; i < n && st == AJC_OK; ++i)
      if ((int64_t)blen[i] < 0) st = AMBRYCRC_EINVAL;
    if (st == AJC_OK && wire_out) st = gather_list(env, fields, n, fp, fl);
    if (st == AJC_OK && record_out) st = gather_list(env, prefixes, n, pp, pl);
    if (st == AJC_OK) {
      for (jsize i = 0; i < n; ++i) {
        fl64[i] = wire_out ? (uint64_t)fl[i] : 0;
        pl64[i] = record_out ? (uint64_t)pl[i] : 0;
      }
      st = ambrycrc_put_crcs((const uint8_t* const*)fp, fl64, (const uint8_t* const*)pp, pl64, crc, blen, (size_t)n,
                             wire_out ? wire : NULL, record_out ? rec : NULL);
    }
    if (st == AJC_OK && wire_out) (*env)->SetIntArrayRegion(env, wire_out, 0, n, (const jint*)wire);
    if (st == AJC_OK && record_out) (*env)->SetIntArrayRegion(env, record_out, 0, n, (const jint*)rec);
  }
  free(crc);
  free(blen);
  free(fp);
  free(fl);
  free(pp);
  free(pl);
  free(fl64);
  free(pl64);
  free(wire);
  free(rec);
  raise(env, st);
}

/* NativeCrc32.rangeChecksums -> ambrycrc_range_checksums_host: FileStore.getChecksumsForRanges
 * (FileStore.java:567-595) over a file image in a direct buffer (a MappedByteBuffer: capacity = file length).
 * out[i] = CRC of [first[i], second[i]) truncated at the image's end; an invalid range throws
 * IllegalArgumentException before anything is computed. A direct buffer of capacity 0 (an empty file's
 * mapping, which has no address) is an empty image. */
JNIEXPORT void JNICALL JNI_FN(nativeRangeChecksums)(JNIEnv* env, jclass cls, jobject file, jlongArray first,
                                                    jlongArray second, jintArray out, jint device) {
  (void)cls;
  if (!file || !first || !second || !out) {
    raise(env, AJC_ENULL);
    return;
  }
  const jsize n = (*env)->GetArrayLength(env, first);
  if (raise(env, ajc_range_lengths(n, (*env)->GetArrayLength(env, second), (*env)->GetArrayLength(env, out)))) return;
  int64_t cap;
  const uint8_t* base = direct(env, file, &cap);
  if (!base) {
    if ((*env)->GetDirectBufferCapacity(env, file) != 0) {
      raise(env, AJC_ENOTDIRECT);
      return;
    }
    cap = 0;
  }
  if (n == 0) return;
  int64_t* f = (int64_t*)malloc(sizeof(int64_t) * (size_t)n);
  int64_t* s = (int64_t*)malloc(sizeof(int64_t) * (size_t)n);
  uint32_t* res = (uint32_t*)malloc(sizeof(uint32_t) * (size_t)n);
  int st = AMBRYCRC_ENOMEM;
  if (f && s && res) {
    (*env)->GetLongArrayRegion(env, first, 0, n, (jlong*)f);
    (*env)->GetLongArrayRegion(env, second, 0, n, (jlong*)s);
    st = ambrycrc_range_checksums_host(base, (uint64_t)cap, f, s, (size_t)n, res, device);
    if (st == AMBRYCRC_OK) (*env)->SetIntArrayRegion(env, out, 0, n, (const jint*)res);
  }
  free(f);
  free(s);
  free(res);
  raise(env, st);
}

/* One message on the CPU (ambrycrc_verify_message_cpu): MessageFormatSend / BlobStoreRecovery's
 * per-message read. Returns the status bits; end[0] = the message end (0: unparseable). */
JNIEXPORT jint JNICALL JNI_FN(nativeVerifyMessage)(JNIEnv* env, jclass cls, jobject region, jlong offset,
                                                   jlongArray end) {
  (void)cls;
  if (!region) return raise(env, AJC_ENULL), 0;
  if (end && (*env)->GetArrayLength(env, end) < 1) return raise(env, AJC_ESHORT), 0;
  if (offset < 0) return raise(env, AJC_EBOUNDS), 0;
  int64_t cap;
  const uint8_t* base = direct(env, region, &cap);
  if (!base) return raise(env, AJC_ENOTDIRECT), 0;
  uint32_t st = 0;
  uint64_t e = 0;
  if (raise(env, ambrycrc_verify_message_cpu(base, (uint64_t)cap, (uint64_t)offset, &st, &e))) return 0;
  if (end) {
    const jlong je = (jlong)e;
    (*env)->SetLongArrayRegion(env, end, 0, 1, &je);
  }
  return (jint)st;
}

/* BlobStoreRecovery's hop from header to header (BlobStoreRecovery.java:43-110) over a log span in
 * a direct buffer -> ambrycrc_chain_messages_host: up to offsets.length message starts from `start`.
 * Returns how many. */
JNIEXPORT jint JNICALL JNI_FN(nativeChainMessages)(JNIEnv* env, jclass cls, jobject region, jlong start,
                                                   jlongArray offsets) {
  (void)cls;
  if (!region || !offsets) return raise(env, AJC_ENULL), 0;
  if (start < 0) return raise(env, AJC_EBOUNDS), 0;
  int64_t cap;
  const uint8_t* base = direct(env, region, &cap);
  if (!base) return raise(env, AJC_ENOTDIRECT), 0;
  const jsize max = (*env)->GetArrayLength(env, offsets);
  if (max == 0 || start >= cap) return 0;
  uint64_t* offs = (uint64_t*)malloc(sizeof(uint64_t) * (size_t)max);
  if (!offs) return raise(env, AMBRYCRC_ENOMEM), 0;
  const size_t n = ambrycrc_chain_messages_host(base, (uint64_t)cap, (uint64_t)start, offs, (size_t)max);
  if (n) (*env)->SetLongArrayRegion(env, offsets, 0, (jsize)n, (const jlong*)offs);
  free(offs);
  return (jint)n;
}

/* ValidatingTransformer.transform for one message (ambrycrc_transform_message_cpu) into the direct
 * buffer `out` from its position 0. Returns the status bits; outLen[0] = bytes written. */
JNIEXPORT jint JNICALL JNI_FN(nativeTransformMessage)(JNIEnv* env, jclass cls, jobject region, jlong offset,
                                                      jint life_version, jint header_version, jobject out,
                                                      jlongArray out_len) {
  (void)cls;
  if (!region || !out || !out_len) return raise(env, AJC_ENULL), 0;
  if ((*env)->GetArrayLength(env, out_len) < 1) return raise(env, AJC_ESHORT), 0;
  if (offset < 0) return raise(env, AJC_EBOUNDS), 0;
  int64_t cap, ocap;
  const uint8_t* base = direct(env, region, &cap);
  uint8_t* dst = (uint8_t*)direct(env, out, &ocap);
  if (!base || !dst) return raise(env, AJC_ENOTDIRECT), 0;
  uint32_t st = 0;
  uint64_t n = 0;
  if (raise(env, ambrycrc_transform_message_cpu(base, (uint64_t)cap, (uint64_t)offset, life_version, header_version,
                                                dst, (uint64_t)ocap, &n, &st)))
    return 0;
  const jlong jn = (jlong)n;
  (*env)->SetLongArrayRegion(env, out_len, 0, 1, &jn);
  return (jint)st;
}

/* ValidatingTransformer.transform over a batch (MessageSievingInputStream.java:130,278-288 over one
 * GetResponse, ReplicaThread.java:1810-1815) -> ambrycrc_transform_messages_host: the messages at
 * `offsets` in the direct buffer `region`, re-serialized at headerVersion with lifeVersions[i]
 * (null: the stored ones), packed in message order into the direct buffer `out` from 0 (its
 * capacity is the output cap: NativeCrc32.transformOutBound sizes it). outOffsets[i] (nullable;
 * -1 when not transformed), outLens[i] and status[i] get the per-message results. */
JNIEXPORT void JNICALL JNI_FN(nativeTransformMessages)(JNIEnv* env, jclass cls, jobject region, jlongArray offsets,
                                                       jshortArray life_versions, jint header_version, jobject out,
                                                       jlongArray out_offsets, jlongArray out_lens, jintArray status,
                                                       jint device) {
  (void)cls;
  if (!region || !offsets || !out || !out_lens || !status) {
    raise(env, AJC_ENULL);
    return;
  }
  const jsize m = (*env)->GetArrayLength(env, offsets);
  if (raise(env, ajc_transform_lengths(m, life_versions ? (*env)->GetArrayLength(env, life_versions) : -1,
                                       out_offsets ? (*env)->GetArrayLength(env, out_offsets) : -1,
                                       (*env)->GetArrayLength(env, out_lens), (*env)->GetArrayLength(env, status))))
    return;
  int64_t cap, ocap;
  const uint8_t* base = direct(env, region, &cap);
  uint8_t* dst = (uint8_t*)direct(env, out, &ocap);
  if (!base || !dst) {
    raise(env, AJC_ENOTDIRECT);
    return;
  }
  if (m == 0) return;
  uint64_t* offs = (uint64_t*)malloc(sizeof(uint64_t) * (size_t)m);
  int16_t* life = life_versions ? (int16_t*)malloc(sizeof(int16_t) * (size_t)m) : NULL;
  uint64_t* oo = (uint64_t*)malloc(sizeof(uint64_t) * (size_t)m);
  uint64_t* ol = (uint64_t*)malloc(sizeof(uint64_t) * (size_t)m);
  uint32_t* st = (uint32_t*)malloc(sizeof(uint32_t) * (size_t)m);
  int rc = AMBRYCRC_ENOMEM;
  if (offs && oo && ol && st && (!life_versions || life)) {
    (*env)->GetLongArrayRegion(env, offsets, 0, m, (jlong*)offs);
    if (life_versions) (*env)->GetShortArrayRegion(env, life_versions, 0, m, (jshort*)life);
    rc = ambrycrc_transform_messages_host(base, (uint64_t)cap, offs, (size_t)m, life, header_version, dst,
                                          (uint64_t)ocap, oo, ol, st, device, 0);
    if (rc == AMBRYCRC_OK) {
      if (out_offsets) (*env)->SetLongArrayRegion(env, out_offsets, 0, m, (const jlong*)oo);
      (*env)->SetLongArrayRegion(env, out_lens, 0, m, (const jlong*)ol);
      (*env)->SetIntArrayRegion(env, status, 0, m, (const jint*)st);
    }
  }
  free(offs);
  free(life);
  free(oo);
  free(ol);
  free(st);
  raise(env, rc);
}

/* NativeCrc32.setHostPolicy: the host-resident dispatch policy of `device` (ambrycrc_set_host_policy:
 * 0 auto, 1 GPU, 2 CPU); returns the previous one. */
JNIEXPORT jint JNICALL JNI_FN(nativeSetHostPolicy)(JNIEnv* env, jclass cls, jint device, jint policy) {
  (void)cls;
  const int r = ambrycrc_set_host_policy(device, policy);
  if (r < 0) return raise(env, r), -1;
  return r;
}

/* NativeCrc32.hostRates: out[0] = the CPU leg's GiB/s, out[1] = the GPU host path's, out[2] = the CPU
 * threads (ambrycrc_host_rates); returns the leg auto takes for pageable bytes (0 CPU, 1 GPU). */
JNIEXPORT jint JNICALL JNI_FN(nativeHostRates)(JNIEnv* env, jclass cls, jint device, jdoubleArray out) {
  (void)cls;
  if (!out) return raise(env, AJC_ENULL), -1;
  if ((*env)->GetArrayLength(env, out) < 3) return raise(env, AJC_ESHORT), -1;
  double cpu = 0, gpu = 0;
  int threads = 0;
  const int r = ambrycrc_host_rates(device, &cpu, &gpu, &threads);
  if (r < 0) return raise(env, r), -1;
  const jdouble v[3] = {cpu, gpu, (jdouble)threads};
  (*env)->SetDoubleArrayRegion(env, out, 0, 3, v);
  return r;
}

/* NativeCrc32.lastHostPath: the leg `device`'s last host-resident call took (0 CPU, 1 GPU, -1 none). */
JNIEXPORT jint JNICALL JNI_FN(nativeLastHostPath)(JNIEnv* env, jclass cls, jint device) {
  (void)cls;
  const int r = ambrycrc_last_host_path(device);
  if (r < -1) return raise(env, r), -1;
  return r;
}

/* NativeCrc32.setHostCpuThreads: the CPU leg's thread budget (ambrycrc_set_host_cpu_threads; device -1: the
 * process's, threads 0: the default); returns the previous one. */
JNIEXPORT jint JNICALL JNI_FN(nativeSetHostCpuThreads)(JNIEnv* env, jclass cls, jint device, jint threads) {
  (void)cls;
  const int r = ambrycrc_set_host_cpu_threads(device, threads);
  if (r < 0) return raise(env, r), -1;
  return r;
}
