/*
 * ambrycrc_jni.c -- JNI shim binding com.github.ambry.utils.NativeCrc32 (see
 * INTEGRATION.md) to libambrycrc's C ABI (include/ambrycrc.h).
 *
 * Built only where a JDK provides jni.h (`make -C ambry_amd jni JAVA_HOME=...`);
 * this build image has no JDK, so the shim is source-only here.
 *
 * Java side it serves:
 *   final class NativeCrc32 implements java.util.zip.Checksum     (drop-in for
 *     ambry-utils/.../utils/Crc32.java:34 and, after retyping, the CRC32 fields of
 *     CrcInputStream.java:28 / CrcOutputStream.java:25)
 *   static native int  nativeUpdateArray(int crc, byte[] b, int off, int len);
 *   static native int  nativeUpdateDirect(int crc, java.nio.ByteBuffer buf, int pos, int len);
 *   static native int  nativeUpdateByte(int crc, int b);
 *   static native int  nativeUpdateDirectAll(int crc, java.nio.ByteBuffer[] bufs);
 *   static native int  nativeCombine(int crc1, int crc2, long len2);
 *   static native int  nativeInit(int device);
 *   static native int  nativeBatchDirect(java.nio.ByteBuffer[] bufs, int[] pos, int[] len,
 *                                        int[] crcIn, int[] out, int device);
 *   static native int  nativeVerifyMessages(java.nio.ByteBuffer region, long[] offsets,
 *                                           int[] status, long[] ends, int device);
 * Errors are returned as negative ints (AMBRYCRC_E*); the Java wrapper maps them
 * to exceptions. CRC values travel as Java ints holding the uint32 bit pattern.
 */
#include <jni.h>
#include <stdint.h>
#include <stdlib.h>

#include "../../include/ambrycrc.h"

#define JNI_FN(name) Java_com_github_ambry_utils_NativeCrc32_##name

JNIEXPORT jint JNICALL JNI_FN(nativeInit)(JNIEnv* env, jclass cls, jint device) {
  (void)env;
  (void)cls;
  return ambrycrc_init(device);
}

/* Crc32.update(byte[] b, int off, int len) -- Crc32.java:55-98. Heap arrays are pinned
 * with GetPrimitiveArrayCritical only for the duration of the host-side update. */
JNIEXPORT jint JNICALL JNI_FN(nativeUpdateArray)(JNIEnv* env, jclass cls, jint crc, jbyteArray b, jint off,
                                                 jint len) {
  (void)cls;
  if (len <= 0) return crc;
  jbyte* p = (jbyte*)(*env)->GetPrimitiveArrayCritical(env, b, NULL);
  if (!p) return crc;
  uint32_t r = ambrycrc_update((uint32_t)crc, (const uint8_t*)p + off, (size_t)len);
  (*env)->ReleasePrimitiveArrayCritical(env, b, p, JNI_ABORT);
  return (jint)r;
}

/* Crc32.update(ByteBuffer) on a direct buffer (Crc32.java:100-143); the Java side
 * then sets position(limit) as the reference method does. */
JNIEXPORT jint JNICALL JNI_FN(nativeUpdateDirect)(JNIEnv* env, jclass cls, jint crc, jobject buf, jint pos,
                                                  jint len) {
  (void)cls;
  if (len <= 0) return crc;
  const uint8_t* p = (const uint8_t*)(*env)->GetDirectBufferAddress(env, buf);
  if (!p) return AMBRYCRC_EINVAL;
  return (jint)ambrycrc_update((uint32_t)crc, p + pos, (size_t)len);
}

/* Crc32.update(int b) -- Crc32.java:146-148. */
JNIEXPORT jint JNICALL JNI_FN(nativeUpdateByte)(JNIEnv* env, jclass cls, jint crc, jint b) {
  (void)env;
  (void)cls;
  return (jint)ambrycrc_update_byte((uint32_t)crc, b);
}

JNIEXPORT jint JNICALL JNI_FN(nativeCombine)(JNIEnv* env, jclass cls, jint crc1, jint crc2, jlong len2) {
  (void)env;
  (void)cls;
  return (jint)ambrycrc_combine((uint32_t)crc1, (uint32_t)crc2, (uint64_t)len2);
}

/* Batch of direct ByteBuffers (Netty nioBuffers / registered arenas) -> device path
 * (ambrycrc_batch_host: pinned staging, hipMemcpyAsync, gfx950 kernels). */
JNIEXPORT jint JNICALL JNI_FN(nativeBatchDirect)(JNIEnv* env, jclass cls, jobjectArray bufs, jintArray pos,
                                                 jintArray len, jintArray crc_in, jintArray out, jint device) {
  (void)cls;
  const jsize n = (*env)->GetArrayLength(env, bufs);
  if (n <= 0) return AMBRYCRC_OK;
  const void** ptrs = (const void**)malloc(sizeof(void*) * (size_t)n);
  uint64_t* lens = (uint64_t*)malloc(sizeof(uint64_t) * (size_t)n);
  uint32_t* cin = crc_in ? (uint32_t*)malloc(sizeof(uint32_t) * (size_t)n) : NULL;
  uint32_t* res = (uint32_t*)malloc(sizeof(uint32_t) * (size_t)n);
  jint rc = AMBRYCRC_ENOMEM;
  if (!ptrs || !lens || !res || (crc_in && !cin)) goto done;
  jint* jpos = (*env)->GetIntArrayElements(env, pos, NULL);
  jint* jlen = (*env)->GetIntArrayElements(env, len, NULL);
  jint* jcin = crc_in ? (*env)->GetIntArrayElements(env, crc_in, NULL) : NULL;
  rc = AMBRYCRC_OK;
  for (jsize i = 0; i < n; ++i) {
    jobject b = (*env)->GetObjectArrayElement(env, bufs, i);
    const uint8_t* base = (const uint8_t*)(*env)->GetDirectBufferAddress(env, b);
    if (!base) rc = AMBRYCRC_EINVAL;
    ptrs[i] = base ? base + jpos[i] : NULL;
    lens[i] = (uint64_t)jlen[i];
    if (cin) cin[i] = (uint32_t)jcin[i];
    (*env)->DeleteLocalRef(env, b);
  }
  (*env)->ReleaseIntArrayElements(env, pos, jpos, JNI_ABORT);
  (*env)->ReleaseIntArrayElements(env, len, jlen, JNI_ABORT);
  if (jcin) (*env)->ReleaseIntArrayElements(env, crc_in, jcin, JNI_ABORT);
  if (rc == AMBRYCRC_OK) rc = ambrycrc_batch_host(ptrs, lens, cin, res, (size_t)n, device, 0);
  if (rc == AMBRYCRC_OK) (*env)->SetIntArrayRegion(env, out, 0, n, (const jint*)res);
done:
  free(ptrs);
  free(lens);
  free(cin);
  free(res);
  return rc;
}

/* Verify every CRC of the PUT / update messages at `offsets` in a direct ByteBuffer holding a
 * log-segment region (BlobStoreRecovery.java:43-110 scan, MessageFormatSend.java:131-139 on
 * GET, ValidatingTransformer.java:46-104 on replication) -> ambrycrc_verify_messages_host.
 * status[i]: AMBRYCRC_MSG_* bits (0 = every CRC matches); ends[i]: message end or 0. */
JNIEXPORT jint JNICALL JNI_FN(nativeVerifyMessages)(JNIEnv* env, jclass cls, jobject region, jlongArray offsets,
                                                    jintArray status, jlongArray ends, jint device) {
  (void)cls;
  const jsize m = (*env)->GetArrayLength(env, offsets);
  if (m <= 0) return AMBRYCRC_OK;
  const uint8_t* base = (const uint8_t*)(*env)->GetDirectBufferAddress(env, region);
  const jlong cap = (*env)->GetDirectBufferCapacity(env, region);
  if (!base || cap < 0 || (*env)->GetArrayLength(env, status) < m ||
      (ends && (*env)->GetArrayLength(env, ends) < m))
    return AMBRYCRC_EINVAL;
  uint64_t* offs = (uint64_t*)malloc(sizeof(uint64_t) * (size_t)m);
  uint32_t* st = (uint32_t*)malloc(sizeof(uint32_t) * (size_t)m);
  uint64_t* en = ends ? (uint64_t*)malloc(sizeof(uint64_t) * (size_t)m) : NULL;
  jint rc = AMBRYCRC_ENOMEM;
  if (offs && st && (!ends || en)) {
    (*env)->GetLongArrayRegion(env, offsets, 0, m, (jlong*)offs);  /* jlong and uint64_t: same width */
    rc = ambrycrc_verify_messages_host(base, (uint64_t)cap, offs, (size_t)m, st, en, device, 0);
    if (rc == AMBRYCRC_OK) {
      (*env)->SetIntArrayRegion(env, status, 0, m, (const jint*)st);
      if (ends) (*env)->SetLongArrayRegion(env, ends, 0, m, (const jlong*)en);
    }
  }
  free(offs);
  free(st);
  free(en);
  return rc;
}

/* The loop of PutOperation.PutChunk.verifyCRC (PutOperation.java:2041-2043) over a Netty
 * CompositeByteBuf's nioBuffers(), all direct: one JNI crossing for the whole gather list
 * (ambrycrc_update_iov). Each buffer's position..limit is used; the Java side consumes them. */
JNIEXPORT jint JNICALL JNI_FN(nativeUpdateDirectAll)(JNIEnv* env, jclass cls, jint crc, jobjectArray bufs) {
  (void)cls;
  const jsize n = (*env)->GetArrayLength(env, bufs);
  if (n <= 0) return crc;
  const void** ptrs = (const void**)malloc(sizeof(void*) * (size_t)n);
  size_t* lens = (size_t*)malloc(sizeof(size_t) * (size_t)n);
  if (!ptrs || !lens) {
    free(ptrs);
    free(lens);
    return crc;  /* the Java wrapper checks isDirect() and sizes; allocation failure: unchanged */
  }
  jclass bbc = (*env)->FindClass(env, "java/nio/Buffer");
  jmethodID mpos = bbc ? (*env)->GetMethodID(env, bbc, "position", "()I") : NULL;
  jmethodID mlim = bbc ? (*env)->GetMethodID(env, bbc, "limit", "()I") : NULL;
  for (jsize i = 0; i < n; ++i) {
    jobject b = (*env)->GetObjectArrayElement(env, bufs, i);
    const uint8_t* base = (const uint8_t*)(*env)->GetDirectBufferAddress(env, b);
    const jint pos = mpos ? (*env)->CallIntMethod(env, b, mpos) : 0;
    const jint lim = mlim ? (*env)->CallIntMethod(env, b, mlim) : 0;
    ptrs[i] = base ? base + pos : NULL;
    lens[i] = (base && lim > pos) ? (size_t)(lim - pos) : 0;
    (*env)->DeleteLocalRef(env, b);
  }
  const jint out = (jint)ambrycrc_update_iov((uint32_t)crc, ptrs, lens, (size_t)n);
  free(ptrs);
  free(lens);
  return out;
}
