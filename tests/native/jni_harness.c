/*
 * A fake JVM for ambry_amd/jni/ambrycrc_jni.c: Java objects are tagged C structs, the JNIEnv a
 * table of the functions the shim calls (tests/native/jni_stub/jni.h). Each case calls a
 * Java_com_github_ambry_utils_NativeCrc32_* entry the way NativeCrc32.java does and prints
 *   <case> <returned int as unsigned hex> <pending exception class or ->
 * for tests/test_jni_core.py to check against zlib and the exception mapping. CPU entries only
 * (no GPU in the build container): nativeInit and the batch / verify entries are driven into
 * their argument errors and, for nativeInit, the no-device error.
 */
#include <jni.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../include/ambrycrc.h"

enum Kind { K_CLASS, K_BYTES, K_INTS, K_LONGS, K_SHORTS, K_OBJS, K_BUFFER, K_DOUBLES };

struct _jobject {
  enum Kind kind;
  jsize len;           /* array length, or buffer capacity */
  void* data;          /* elements, or the direct buffer's address (NULL: heap buffer) */
  jint pos, lim;       /* ByteBuffer position / limit */
  const char* name;    /* class name */
};

static char g_exc[256];
static int g_pending;
static struct _jobject g_classes[8];
static int g_nclasses;
static struct _jmethodID {
  int which;
} g_mpos = {0}, g_mlim = {1};

static jclass find_class(JNIEnv* env, const char* name) {
  (void)env;
  struct _jobject* c = &g_classes[g_nclasses++ % 8];
  c->kind = K_CLASS;
  c->name = name;
  return c;
}
static jint throw_new(JNIEnv* env, jclass cls, const char* msg) {
  (void)env;
  (void)msg;
  if (!g_pending) snprintf(g_exc, sizeof g_exc, "%s", cls->name);
  g_pending = 1;
  return 0;
}
static jboolean exception_check(JNIEnv* env) {
  (void)env;
  return (jboolean)g_pending;
}
static void delete_local_ref(JNIEnv* env, jobject o) {
  (void)env;
  (void)o;
}
static jmethodID get_method_id(JNIEnv* env, jclass c, const char* name, const char* sig) {
  (void)env;
  (void)c;
  (void)sig;
  return strcmp(name, "position") == 0 ? &g_mpos : strcmp(name, "limit") == 0 ? &g_mlim : NULL;
}
static jint call_int_method(JNIEnv* env, jobject o, jmethodID m, ...) {
  (void)env;
  return m->which == 0 ? o->pos : o->lim;
}
static jsize get_array_length(JNIEnv* env, jarray a) {
  (void)env;
  return a->len;
}
static jobject get_object_array_element(JNIEnv* env, jobjectArray a, jsize i) {
  (void)env;
  if (i < 0 || i >= a->len) abort(); /* a JVM would throw; the shim must never ask */
  return ((jobject*)a->data)[i];
}
static void region_check(jarray a, jsize start, jsize len) {
  if (start < 0 || len < 0 || start + len > a->len) abort();
}
static void get_int_region(JNIEnv* env, jintArray a, jsize s, jsize n, jint* buf) {
  (void)env;
  region_check(a, s, n);
  memcpy(buf, (jint*)a->data + s, sizeof(jint) * (size_t)n);
}
static void set_int_region(JNIEnv* env, jintArray a, jsize s, jsize n, const jint* buf) {
  (void)env;
  region_check(a, s, n);
  memcpy((jint*)a->data + s, buf, sizeof(jint) * (size_t)n);
}
static void get_long_region(JNIEnv* env, jlongArray a, jsize s, jsize n, jlong* buf) {
  (void)env;
  region_check(a, s, n);
  memcpy(buf, (jlong*)a->data + s, sizeof(jlong) * (size_t)n);
}
static void set_long_region(JNIEnv* env, jlongArray a, jsize s, jsize n, const jlong* buf) {
  (void)env;
  region_check(a, s, n);
  memcpy((jlong*)a->data + s, buf, sizeof(jlong) * (size_t)n);
}
static void get_short_region(JNIEnv* env, jshortArray a, jsize s, jsize n, jshort* buf) {
  (void)env;
  region_check(a, s, n);
  memcpy(buf, (jshort*)a->data + s, sizeof(jshort) * (size_t)n);
}
static void* get_critical(JNIEnv* env, jarray a, jboolean* copy) {
  (void)env;
  if (copy) *copy = JNI_FALSE;
  return a->data;
}
static void release_critical(JNIEnv* env, jarray a, void* p, jint mode) {
  (void)env;
  (void)a;
  (void)p;
  (void)mode;
}
static void* direct_address(JNIEnv* env, jobject b) {
  (void)env;
  return b->kind == K_BUFFER ? b->data : NULL;
}
static jlong direct_capacity(JNIEnv* env, jobject b) {
  (void)env;
  return b->kind == K_BUFFER && b->data ? b->len : -1;
}

static void set_double_region(JNIEnv* env, jdoubleArray a, jsize s, jsize n, const jdouble* buf) {
  (void)env;
  region_check(a, s, n);
  memcpy((jdouble*)a->data + s, buf, (size_t)n * sizeof(jdouble));
}
static const struct JNINativeInterface_ g_fns = {
    find_class,         throw_new,       exception_check, delete_local_ref, get_method_id,
    call_int_method,    get_array_length, get_object_array_element, get_int_region, set_int_region,
    get_long_region,    set_long_region, get_short_region, get_critical,   release_critical,
    direct_address,     direct_capacity, set_double_region,
};
static JNIEnv g_env = &g_fns;

#define FN(name) Java_com_github_ambry_utils_NativeCrc32_##name
JNIEXPORT void JNICALL FN(nativeInit)(JNIEnv*, jclass, jint);
JNIEXPORT jint JNICALL FN(nativeUpdateArray)(JNIEnv*, jclass, jint, jbyteArray, jint, jint);
JNIEXPORT jint JNICALL FN(nativeUpdateDirect)(JNIEnv*, jclass, jint, jobject, jint, jint);
JNIEXPORT jint JNICALL FN(nativeUpdateByte)(JNIEnv*, jclass, jint, jint);
JNIEXPORT jint JNICALL FN(nativeCombine)(JNIEnv*, jclass, jint, jint, jlong);
JNIEXPORT jint JNICALL FN(nativeUpdateDirectAll)(JNIEnv*, jclass, jint, jobjectArray);
JNIEXPORT void JNICALL FN(nativeBatchDirect)(JNIEnv*, jclass, jobjectArray, jintArray, jintArray, jintArray,
                                             jintArray, jint);
JNIEXPORT void JNICALL FN(nativeVerifyMessages)(JNIEnv*, jclass, jobject, jlongArray, jintArray, jlongArray, jint);

static void report(const char* name, jint r) {
  printf("%s %08x %s\n", name, (unsigned)r, g_pending ? g_exc : "-");
  g_pending = 0;
  g_exc[0] = 0;
}

static struct _jobject arr(enum Kind k, void* data, jsize len) {
  struct _jobject o;
  memset(&o, 0, sizeof o);
  o.kind = k;
  o.data = data;
  o.len = len;
  return o;
}

JNIEXPORT jint JNICALL FN(nativeVerifyMessage)(JNIEnv*, jclass, jobject, jlong, jlongArray);
JNIEXPORT jint JNICALL FN(nativeTransformMessage)(JNIEnv*, jclass, jobject, jlong, jint, jint, jobject, jlongArray);
JNIEXPORT void JNICALL FN(nativeTransformMessages)(JNIEnv*, jclass, jobject, jlongArray, jshortArray, jint, jobject,
                                                   jlongArray, jlongArray, jintArray, jint);

/* argv[1] == "gpumsg", argv[2] = one PUT message (header V3, properties at SerDe V5): the batched
 * transform over a region holding it twice, on the GPU. */
static int gpumsg_cases(const char* path) {
  FILE* f = fopen(path, "rb");
  if (!f) return 2;
  static uint8_t region[2 << 20], out[2 << 20];
  const size_t n = fread(region, 1, 1 << 20, f);
  fclose(f);
  memcpy(region + n, region, n);
  FN(nativeInit)(&g_env, NULL, 0);
  report("gpumsg_init", 0);
  struct _jobject reg = arr(K_BUFFER, region, (jsize)(2 * n)), dst = arr(K_BUFFER, out, (jsize)(2 * n + 52));
  jlong offs[2] = {0, (jlong)n}, oo[2] = {-5, -5}, ol[2] = {-5, -5};
  jshort life[2] = {0, 0};
  jint st[2] = {-5, -5};
  struct _jobject joffs = arr(K_LONGS, offs, 2), joo = arr(K_LONGS, oo, 2), jol = arr(K_LONGS, ol, 2);
  struct _jobject jlife = arr(K_SHORTS, life, 2), jst = arr(K_INTS, st, 2);
  FN(nativeTransformMessages)(&g_env, NULL, &reg, &joffs, &jlife, 3, &dst, &joo, &jol, &jst, 0);
  report("gpumsg_xform_st", st[0] | st[1]);
  report("gpumsg_xform_off1", (jint)oo[1]);
  report("gpumsg_xform_len", (jint)(ol[0] + ol[1]));
  report("gpumsg_xform_same", (jint)(memcmp(out, region, 2 * n) == 0));
  /* no room for the second message: cap = one message */
  struct _jobject one = arr(K_BUFFER, out, (jsize)n);
  FN(nativeTransformMessages)(&g_env, NULL, &reg, &joffs, NULL, 3, &one, NULL, &jol, &jst, 0);
  report("gpumsg_xform_room0", st[0]);
  report("gpumsg_xform_room1", st[1]);
  return 0;
}

/* argv[1] == "msg", argv[2] = a file holding one PUT message: the per-message CPU entries. */
static int msg_cases(const char* path) {
  FILE* f = fopen(path, "rb");
  if (!f) return 2;
  static uint8_t msg[1 << 20], out[1 << 20];
  const size_t n = fread(msg, 1, sizeof msg, f);
  fclose(f);
  struct _jobject reg = arr(K_BUFFER, msg, (jsize)n), heap = arr(K_BUFFER, NULL, (jsize)n);
  struct _jobject dst = arr(K_BUFFER, out, (jsize)sizeof out), small = arr(K_BUFFER, out, 16);
  jlong end[1] = {-1}, olen[1] = {-1};
  struct _jobject jend = arr(K_LONGS, end, 1), jolen = arr(K_LONGS, olen, 1), jnone = arr(K_LONGS, end, 0);
  report("msg_verify", FN(nativeVerifyMessage)(&g_env, NULL, &reg, 0, &jend));
  report("msg_verify_end", (jint)end[0]);
  report("msg_verify_heap", FN(nativeVerifyMessage)(&g_env, NULL, &heap, 0, &jend));
  report("msg_verify_null", FN(nativeVerifyMessage)(&g_env, NULL, NULL, 0, &jend));
  report("msg_verify_short", FN(nativeVerifyMessage)(&g_env, NULL, &reg, 0, &jnone));
  report("msg_verify_past", FN(nativeVerifyMessage)(&g_env, NULL, &reg, (jlong)n + 5, NULL));
  report("msg_transform_v3", FN(nativeTransformMessage)(&g_env, NULL, &reg, 0, -1, 3, &dst, &jolen));
  report("msg_transform_v3_len", (jint)olen[0]);
  report("msg_transform_v3_same", (jint)(olen[0] == (jlong)n && memcmp(out, msg, n) == 0));
  report("msg_transform_v1", FN(nativeTransformMessage)(&g_env, NULL, &reg, 0, -1, 1, &dst, &jolen));
  report("msg_transform_v1_len", (jint)olen[0]);
  report("msg_transform_small", FN(nativeTransformMessage)(&g_env, NULL, &reg, 0, -1, 3, &small, &jolen));
  report("msg_transform_small_len", (jint)olen[0]);
  report("msg_transform_badver", FN(nativeTransformMessage)(&g_env, NULL, &reg, 0, -1, 7, &dst, &jolen));
  msg[n / 2] ^= 0x20; /* inside the blob content */
  report("msg_verify_corrupt", FN(nativeVerifyMessage)(&g_env, NULL, &reg, 0, &jend));
  report("msg_transform_corrupt", FN(nativeTransformMessage)(&g_env, NULL, &reg, 0, -1, 3, &dst, &jolen));
  return 0;
}

JNIEXPORT jint JNICALL FN(nativeChainMessages)(JNIEnv*, jclass, jobject, jlong, jlongArray);
JNIEXPORT jint JNICALL FN(nativeSetHostPolicy)(JNIEnv*, jclass, jint, jint);
JNIEXPORT jint JNICALL FN(nativeHostRates)(JNIEnv*, jclass, jint, jdoubleArray);
JNIEXPORT jint JNICALL FN(nativeLastHostPath)(JNIEnv*, jclass, jint);
JNIEXPORT jint JNICALL FN(nativeSetHostCpuThreads)(JNIEnv*, jclass, jint, jint);

static uint8_t* slurp(const char* path, size_t* n) {
  FILE* f = fopen(path, "rb");
  if (!f) return NULL;
  fseek(f, 0, SEEK_END);
  const long len = ftell(f);
  fseek(f, 0, SEEK_SET);
  uint8_t* b = (uint8_t*)malloc((len > 0 ? (size_t)len : 0) + 1); /* NUL-terminated: putcrcs_cases scans text */
  *n = b ? fread(b, 1, (size_t)len, f) : 0;
  if (b) b[*n] = 0;
  fclose(f);
  return b;
}

/* argv[1] == "sieve", argv[2] = one GetResponse's bytes, argv[3] = its message infos, one line each:
 * "<size> <flag> <lifeVersion>" (flag 0 live, 1 deleted, 2 expired). The call sequence of
 * MessageSievingInputStream with ambry-messageformat-batch-sieve.patch: every message in one direct
 * buffer, NativeValidatingTransformer.transformAll -> NativeCrc32.transformMessages over the live
 * ones at their response offsets (header V3), then applyOutput per message. Prints per message
 * sieve_<i>: 0 skipped (deleted / expired), 1 sieved (then sieve_<i>_len and sieve_<i>_crc of its
 * output bytes), 2 invalid (MessageFormatException: skipped, counted), 3 fatal (the exception that
 * fails the stream: an update record, a property string the V5 re-encoding cannot hold). */
static int sieve_cases(const char* rpath, const char* mpath) {
  size_t rn = 0;
  uint8_t* region = slurp(rpath, &rn);
  FILE* f = fopen(mpath, "r");
  if (!region || !f) return 2;
  static jlong offs[4096], oo[4096], ol[4096];
  static int flag[4096];
  static jshort life[4096];
  static jint st[4096];
  int n = 0, m = 0;
  long long sz;
  int fl, lv;
  jlong at = 0, live_bytes = 0;
  while (n < 4096 && fscanf(f, "%lld %d %d", &sz, &fl, &lv) == 3) {
    flag[n] = fl;
    if (fl == 0) {  /* transformAll: live messages at their offsets in the response */
      offs[m] = at;
      life[m] = (jshort)lv;
      live_bytes += sz;
      ++m;
    }
    at += sz;
    ++n;
  }
  fclose(f);
  if ((size_t)at > rn) return 3;
  const jlong cap = live_bytes + 26 * (jlong)m; /* NativeCrc32.transformOutBound(bytes, m) */
  uint8_t* out = (uint8_t*)malloc((size_t)cap + 1);
  FN(nativeInit)(&g_env, NULL, 0);
  report("sieve_init", 0);
  struct _jobject reg = arr(K_BUFFER, region, (jsize)rn), dst = arr(K_BUFFER, out, (jsize)cap);
  struct _jobject joffs = arr(K_LONGS, offs, m), jlife = arr(K_SHORTS, life, m), joo = arr(K_LONGS, oo, m);
  struct _jobject jol = arr(K_LONGS, ol, m), jst = arr(K_INTS, st, m);
  FN(nativeTransformMessages)(&g_env, NULL, &reg, &joffs, &jlife, 3, &dst, &joo, &jol, &jst, 0);
  report("sieve_transform", 0);
  int k = 0;
  char name[64];
  for (int i = 0; i < n; ++i) {
    snprintf(name, sizeof name, "sieve_%d", i);
    if (flag[i] != 0) {
      report(name, 0);
      continue;
    }
    const uint32_t s = (uint32_t)st[k];
    const jlong off = offs[k];
    ++k;
    if (s == 0) {
      report(name, 1);
      snprintf(name, sizeof name, "sieve_%d_len", i);
      report(name, (jint)ol[k - 1]);
      snprintf(name, sizeof name, "sieve_%d_crc", i);
      report(name, (jint)ambrycrc_update(0, out + oo[k - 1], (size_t)ol[k - 1]));
      continue;
    }
    /* NativeValidatingTransformer.exceptionFor's classes, in its order of checks */
    const int v = (int16_t)((region[off] << 8) | region[off + 1]);
    int cls = 2;
    if (v >= 1 && v <= 3 && !(s & AMBRYCRC_MSG_HEADER_CRC) && !(s & AMBRYCRC_MSG_BAD_LAYOUT)) {
      const uint8_t* u = region + off + (v == 1 ? 14 : v == 2 ? 18 : 20);
      const int32_t upd = (int32_t)(((uint32_t)u[0] << 24) | ((uint32_t)u[1] << 16) | ((uint32_t)u[2] << 8) | u[3]);
      const uint32_t recs = AMBRYCRC_MSG_ENCKEY_CRC | AMBRYCRC_MSG_PROPS_CRC | AMBRYCRC_MSG_USERMETA_CRC |
                            AMBRYCRC_MSG_BLOB_CRC | AMBRYCRC_MSG_BAD_VERSION | AMBRYCRC_MSG_BAD_RECORD;
      if ((s & AMBRYCRC_MSG_NOT_PUT) || upd != -1) cls = 3;
      else if (s & recs) cls = 2;
      else cls = 3; /* NOT_ENCODABLE (BufferOverflowException) or an unknown bit */
    }
    report(name, cls);
  }
  free(out);
  free(region);
  return 0;
}

/* argv[1] == "recover", argv[2] = a log span: the call sequence of NativeBlobStoreRecovery.recover
 * (BlobStoreRecovery.recover with ambry-messageformat-batch-recovery.patch): chainMessages from the
 * span's start in batches of argv[3] offsets, verifyMessages on each batch, the first failing message
 * (or the first header the chain cannot follow) stopping the scan. Prints recover_count (messages
 * recovered), recover_stop (the startOffset the result reports) and recover_failed (1: a
 * LogFileFormatError). */
static int recover_cases(const char* rpath, int batch) {
  size_t rn = 0;
  uint8_t* region = slurp(rpath, &rn);
  if (!region || batch < 1 || batch > 65536) return 2;
  FN(nativeInit)(&g_env, NULL, 0);
  report("recover_init", 0);
  static jlong offs[65536], ends[65536];
  static jint st[65536];
  struct _jobject reg = arr(K_BUFFER, region, (jsize)rn);
  jlong pos = 0;
  int count = 0, failed = 0;
  while (pos < (jlong)rn && !failed) {
    struct _jobject joffs = arr(K_LONGS, offs, batch);
    const jint n = FN(nativeChainMessages)(&g_env, NULL, &reg, pos, &joffs);
    if (g_pending) return 4;
    if (n == 0) {
      failed = 1;
      break;
    }
    struct _jobject jo = arr(K_LONGS, offs, n), js = arr(K_INTS, st, n), je = arr(K_LONGS, ends, n);
    FN(nativeVerifyMessages)(&g_env, NULL, &reg, &jo, &js, &je, 0);
    if (g_pending) return 5;
    for (int k = 0; k < n; ++k) {
      if (st[k] != 0) {
        failed = 1;
        break;
      }
      ++count;
      pos = ends[k];
    }
  }
  report("recover_count", count);
  report("recover_stop", (jint)pos);
  report("recover_failed", failed);
  free(region);
  return 0;
}

JNIEXPORT void JNICALL FN(nativePutCrcs)(JNIEnv*, jclass, jobjectArray, jobjectArray, jintArray, jlongArray, jintArray,
                                         jintArray);
JNIEXPORT void JNICALL FN(nativeRangeChecksums)(JNIEnv*, jclass, jobject, jlongArray, jlongArray, jintArray, jint);

/* com.github.ambry.utils.Crc32 with ambry-utils-crc32-native.patch: the register is kept inverted, updates of at
 * least min_bytes go through NativeCrc32.updateBuffer (nativeUpdateDirect on a direct buffer, which is then
 * consumed), shorter ones through the class's own table loop (Crc32.java:77-94, byte-wise). */
struct crc32_obj {
  jint crc;
};
static uint32_t g_t0[256];
static void crc32_reset(struct crc32_obj* c) { c->crc = (jint)0xffffffffu; }
static void crc32_update_buffer(struct crc32_obj* c, struct _jobject* buf, int min_bytes) {
  const jint len = buf->lim - buf->pos;
  if (len == 0) return;
  if (len >= min_bytes) {
    c->crc = ~FN(nativeUpdateDirect)(&g_env, NULL, ~c->crc, buf, buf->pos, len);
    if (!g_pending) buf->pos = buf->lim;
    return;
  }
  uint32_t r = (uint32_t)c->crc;
  for (; buf->pos < buf->lim; ++buf->pos) r = (r >> 8) ^ g_t0[(r ^ ((const uint8_t*)buf->data)[buf->pos]) & 0xff];
  c->crc = (jint)r;
}
static jint crc32_value(const struct crc32_obj* c) { return ~c->crc; }

/* argv[1] == "putchunk", argv[2] = a chunk's bytes, argv[3..] = the lengths of the slices fillFrom receives: the
 * PutChunk call sequence of PutOperation.java with the patched Crc32 (min_bytes 256). fillFrom updates chunkCrc32
 * with each slice's nioBuffer (:1700-1703); verifyCRC runs a fresh Crc32 over buf.nioBuffers() (:2033-2054) -- the
 * composite's components, here the same slices; a byte mutated after the fill (PutOperationTest.java:629-679) must
 * then fail the comparison; a compressed chunk resets chunkCrc32 and recomputes it over the new buffer
 * (:1595-1599). Prints fill / verify values and the verify outcomes. */
static int putchunk_cases(const char* path, int nslices, char** slices) {
  for (uint32_t i = 0; i < 256; ++i) {
    uint32_t r = i;
    for (int k = 0; k < 8; ++k) r = (r >> 1) ^ (0xEDB88320u & (0u - (r & 1)));
    g_t0[i] = r;
  }
  size_t n = 0;
  uint8_t* chunk = slurp(path, &n);
  if (!chunk || nslices > 256) return 2;
  static struct _jobject bufs[256];
  size_t at = 0;
  for (int i = 0; i < nslices; ++i) {
    const size_t len = (size_t)atol(slices[i]);
    if (at + len > n) return 3;
    bufs[i] = arr(K_BUFFER, chunk + at, (jsize)len); /* slice.nioBuffer(): a direct buffer over the slice */
    bufs[i].pos = 0, bufs[i].lim = (jint)len;
    at += len;
  }
  struct crc32_obj chunk_crc, computed;
  crc32_reset(&chunk_crc);
  for (int i = 0; i < nslices; ++i) crc32_update_buffer(&chunk_crc, &bufs[i], 256); /* fillFrom */
  report("putchunk_fill", crc32_value(&chunk_crc));
  report("putchunk_fill_consumed", bufs[0].pos == bufs[0].lim && bufs[nslices - 1].pos == bufs[nslices - 1].lim);
  /* verifyCRC: buf.nioBuffers() hands out fresh buffers over the components */
  crc32_reset(&computed);
  for (int i = 0; i < nslices; ++i) {
    bufs[i].pos = 0;
    crc32_update_buffer(&computed, &bufs[i], 256);
  }
  report("putchunk_verify", crc32_value(&computed));
  report("putchunk_verify_match", crc32_value(&computed) == crc32_value(&chunk_crc));
  chunk[n / 2] ^= 0x10; /* the buffer mutated after the fill */
  crc32_reset(&computed);
  for (int i = 0; i < nslices; ++i) {
    bufs[i].pos = 0;
    crc32_update_buffer(&computed, &bufs[i], 256);
  }
  report("putchunk_mutated_match", crc32_value(&computed) == crc32_value(&chunk_crc));
  /* compression: chunkCrc32.reset(), then the compressed buffer's nioBuffers (one direct buffer here) */
  struct _jobject whole = arr(K_BUFFER, chunk, (jsize)n);
  whole.pos = 0, whole.lim = (jint)n;
  crc32_reset(&chunk_crc);
  crc32_update_buffer(&chunk_crc, &whole, 256);
  report("putchunk_recomputed", crc32_value(&chunk_crc));
  free(chunk);
  return 0;
}

/* argv[1] == "ranges", argv[2] = a file image, argv[3] = ranges "first second" per line, argv[4] = the device (-1 the
 * CPU): FileStore.getChecksumsForRanges with ambry-store-filestore-ranges.patch -- NativeCrc32.rangeChecksums over a
 * mapping of the file. Prints range_<i> per range (or the exception). An empty file image is a capacity-0 direct
 * buffer. */
static int ranges_cases(const char* fpath, const char* rpath, int device) {
  size_t n = 0;
  uint8_t* image = slurp(fpath, &n);
  FILE* f = fopen(rpath, "r");
  if (!image || !f) return 2;
  static jlong first[4096], second[4096];
  static jint out[4096];
  int k = 0;
  long long a, b;
  while (k < 4096 && fscanf(f, "%lld %lld", &a, &b) == 2) first[k] = a, second[k] = b, ++k;
  fclose(f);
  if (device >= 0) {
    FN(nativeInit)(&g_env, NULL, device);
    report("ranges_init", 0);
  }
  struct _jobject file = arr(K_BUFFER, image, (jsize)n);
  struct _jobject jf = arr(K_LONGS, first, k), js = arr(K_LONGS, second, k), jo = arr(K_INTS, out, k);
  for (int i = 0; i < k; ++i) out[i] = 0x5a5a5a5a;
  FN(nativeRangeChecksums)(&g_env, NULL, &file, &jf, &js, &jo, device);
  report("ranges_call", 0);
  char name[64];
  for (int i = 0; i < k; ++i) {
    snprintf(name, sizeof name, "range_%d", i);
    report(name, out[i]);
  }
  /* argument errors: a short output array, a heap buffer, a null list */
  struct _jobject jshort = arr(K_INTS, out, k > 0 ? k - 1 : 0), heap = arr(K_BUFFER, NULL, (jsize)n);
  if (k > 0) {
    FN(nativeRangeChecksums)(&g_env, NULL, &file, &jf, &js, &jshort, device);
    report("ranges_short", 0);
  }
  FN(nativeRangeChecksums)(&g_env, NULL, &heap, &jf, &js, &jo, device);
  report("ranges_heap", 0);
  FN(nativeRangeChecksums)(&g_env, NULL, &file, NULL, &js, &jo, device);
  report("ranges_null", 0);
  free(image);
  return 0;
}

/* argv[1] == "putcrcs", argv[2] = a file of PUTs, each "<fields len> <prefix len> <blob len>\n" then those bytes:
 * NativeCrc32.putCrcs -- the blob CRCs first (nativeUpdateDirect over each blob), then both CRCs of every PUT from
 * them (ambrycrc_put_crcs: no blob byte read). Prints wire_<i> and record_<i>, then the argument errors. */
static int putcrcs_cases(const char* path) {
  size_t n = 0;
  uint8_t* data = slurp(path, &n);
  if (!data) return 2;
  static struct _jobject fb[512], pb[512];
  static jobject fl[512], pl[512];
  static jint bcrc[512], wire[512], rec[512];
  static jlong blen[512];
  int k = 0;
  size_t at = 0;
  while (at < n && k < 512) {
    unsigned long long a, b, c;
    int used = 0;
    if (sscanf((const char*)data + at, "%llu %llu %llu%n", &a, &b, &c, &used) != 3) return 3;
    at += (size_t)used + 1; /* the newline */
    fb[k] = arr(K_BUFFER, data + at, (jsize)a), fb[k].pos = 0, fb[k].lim = (jint)a;
    pb[k] = arr(K_BUFFER, data + at + a, (jsize)b), pb[k].pos = 0, pb[k].lim = (jint)b;
    struct _jobject blob = arr(K_BUFFER, data + at + a + b, (jsize)c);
    bcrc[k] = c ? FN(nativeUpdateDirect)(&g_env, NULL, 0, &blob, 0, (jint)c) : 0;
    blen[k] = (jlong)c;
    fl[k] = &fb[k], pl[k] = &pb[k];
    at += a + b + c;
    ++k;
  }
  struct _jobject jfl = arr(K_OBJS, fl, k), jpl = arr(K_OBJS, pl, k), jcrc = arr(K_INTS, bcrc, k);
  struct _jobject jlen = arr(K_LONGS, blen, k), jw = arr(K_INTS, wire, k), jr = arr(K_INTS, rec, k);
  FN(nativePutCrcs)(&g_env, NULL, &jfl, &jpl, &jcrc, &jlen, &jw, &jr);
  report("putcrcs_call", 0);
  char name[64];
  for (int i = 0; i < k; ++i) {
    snprintf(name, sizeof name, "wire_%d", i);
    report(name, wire[i]);
    snprintf(name, sizeof name, "record_%d", i);
    report(name, rec[i]);
  }
  /* the record CRCs alone (no field list), then the argument errors */
  for (int i = 0; i < k; ++i) rec[i] = 0;
  FN(nativePutCrcs)(&g_env, NULL, NULL, &jpl, &jcrc, &jlen, NULL, &jr);
  report("putcrcs_record_only_0", rec[0]);
  FN(nativePutCrcs)(&g_env, NULL, NULL, &jpl, &jcrc, &jlen, &jw, &jr);
  report("putcrcs_wire_without_fields", 0);
  struct _jobject jshort = arr(K_INTS, wire, k - 1);
  FN(nativePutCrcs)(&g_env, NULL, &jfl, &jpl, &jcrc, &jlen, &jshort, &jr);
  report("putcrcs_short_out", 0);
  blen[0] = -1;
  FN(nativePutCrcs)(&g_env, NULL, &jfl, &jpl, &jcrc, &jlen, &jw, &jr);
  report("putcrcs_negative_len", 0);
  blen[0] = 0;
  struct _jobject heap = arr(K_BUFFER, NULL, 4);
  fl[0] = &heap;
  FN(nativePutCrcs)(&g_env, NULL, &jfl, &jpl, &jcrc, &jlen, &jw, &jr);
  report("putcrcs_heap_field", 0);
  fb[1].lim = fb[1].len + 1;
  fl[0] = &fb[0];
  FN(nativePutCrcs)(&g_env, NULL, &jfl, &jpl, &jcrc, &jlen, &jw, &jr);
  report("putcrcs_field_bounds", 0);
  free(data);
  return 0;
}

/* With a GPU (argv[1] == "gpu"): the device entries on valid arguments. */
static int gpu_cases(void) {
  FN(nativeInit)(&g_env, NULL, 0);
  report("gpu_init", 0);
  static uint8_t s1[] = "123", s2[] = "xx456", s3[] = "789yy", region[] = "123456789";
  struct _jobject g1 = arr(K_BUFFER, s1, 3), g2 = arr(K_BUFFER, s2, 5), g3 = arr(K_BUFFER, s3, 5);
  jobject list[3] = {&g1, &g2, &g3};
  struct _jobject lst = arr(K_OBJS, list, 3);
  jint pos[3] = {0, 2, 1}, len[3] = {3, 3, 4}, cin[3] = {0, 0, 0}, out[3] = {0, 0, 0};
  struct _jobject jpos = arr(K_INTS, pos, 3), jlen = arr(K_INTS, len, 3), jcin = arr(K_INTS, cin, 3);
  struct _jobject jout = arr(K_INTS, out, 3);
  FN(nativeBatchDirect)(&g_env, NULL, &lst, &jpos, &jlen, &jcin, &jout, 0);
  report("gpu_batch_0", out[0]);
  report("gpu_batch_1", out[1]);
  report("gpu_batch_2", out[2]);
  struct _jobject reg = arr(K_BUFFER, region, 9);
  jlong offs[2] = {0, 4}, ends[2] = {7, 7};
  jint st[2] = {0, 0};
  struct _jobject joffs = arr(K_LONGS, offs, 2), jst = arr(K_INTS, st, 2), jends = arr(K_LONGS, ends, 2);
  FN(nativeVerifyMessages)(&g_env, NULL, &reg, &joffs, &jst, &jends, 0);
  report("gpu_verify_0", st[0]);
  report("gpu_verify_1", st[1]);
  report("gpu_verify_end", (jint)(ends[0] + ends[1]));
  /* host-resident dispatch: the rates auto compares, then the batch above on each forced leg */
  jdouble rates[3] = {0, 0, 0};
  struct _jobject jrates = arr(K_DOUBLES, rates, 3);
  report("gpu_rates_leg", FN(nativeHostRates)(&g_env, NULL, 0, &jrates));
  report("gpu_rates_positive", rates[0] > 0 && rates[1] > 0 && rates[2] >= 1);
  report("gpu_policy_bad", FN(nativeSetHostPolicy)(&g_env, NULL, 0, 7));
  const jint prev = FN(nativeSetHostPolicy)(&g_env, NULL, 0, 2);
  report("gpu_policy_cpu", prev >= 0 && prev <= 2);
  out[0] = out[1] = out[2] = 0;
  FN(nativeBatchDirect)(&g_env, NULL, &lst, &jpos, &jlen, &jcin, &jout, 0);
  report("gpu_cpu_leg_batch_1", out[1]);
  report("gpu_cpu_leg_path", FN(nativeLastHostPath)(&g_env, NULL, 0));
  report("gpu_policy_gpu", FN(nativeSetHostPolicy)(&g_env, NULL, 0, 1));
  out[0] = out[1] = out[2] = 0;
  FN(nativeBatchDirect)(&g_env, NULL, &lst, &jpos, &jlen, &jcin, &jout, 0);
  report("gpu_gpu_leg_batch_1", out[1]);
  report("gpu_gpu_leg_path", FN(nativeLastHostPath)(&g_env, NULL, 0));
  FN(nativeSetHostPolicy)(&g_env, NULL, 0, prev);
  return 0;
}

int main(int argc, char** argv) {
  if (argc > 1 && strcmp(argv[1], "gpu") == 0) return gpu_cases();
  if (argc > 2 && strcmp(argv[1], "msg") == 0) return msg_cases(argv[2]);
  if (argc > 2 && strcmp(argv[1], "gpumsg") == 0) return gpumsg_cases(argv[2]);
  if (argc > 3 && strcmp(argv[1], "sieve") == 0) return sieve_cases(argv[2], argv[3]);
  if (argc > 3 && strcmp(argv[1], "recover") == 0) return recover_cases(argv[2], atoi(argv[3]));
  if (argc > 3 && strcmp(argv[1], "putchunk") == 0) return putchunk_cases(argv[2], argc - 3, argv + 3);
  if (argc > 4 && strcmp(argv[1], "ranges") == 0) return ranges_cases(argv[2], argv[3], atoi(argv[4]));
  if (argc > 2 && strcmp(argv[1], "putcrcs") == 0) return putcrcs_cases(argv[2]);
  static uint8_t digits[] = "123456789";
  struct _jobject b9 = arr(K_BYTES, digits, 9);
  report("array_full", FN(nativeUpdateArray)(&g_env, NULL, 0, &b9, 0, 9));
  report("array_tail", FN(nativeUpdateArray)(&g_env, NULL, 0, &b9, 4, 5));
  report("array_bounds", FN(nativeUpdateArray)(&g_env, NULL, 0x1234, &b9, 5, 5));
  report("array_negative", FN(nativeUpdateArray)(&g_env, NULL, 0x1234, &b9, -1, 2));
  report("array_null", FN(nativeUpdateArray)(&g_env, NULL, 0x1234, NULL, 0, 0));

  struct _jobject direct_buf = arr(K_BUFFER, digits, 9);
  struct _jobject heap_buf = arr(K_BUFFER, NULL, 9);
  report("direct_full", FN(nativeUpdateDirect)(&g_env, NULL, 0, &direct_buf, 0, 9));
  report("direct_bounds", FN(nativeUpdateDirect)(&g_env, NULL, 7, &direct_buf, 8, 2));
  report("direct_heap", FN(nativeUpdateDirect)(&g_env, NULL, 7, &heap_buf, 0, 1));
  report("direct_null", FN(nativeUpdateDirect)(&g_env, NULL, 7, NULL, 0, 1));

  report("byte", FN(nativeUpdateByte)(&g_env, NULL, 0, '1'));
  /* crc("1234") = 0x9be3e0a3, crc("56789") = 0x131da070 (zlib) */
  report("combine", FN(nativeCombine)(&g_env, NULL, (jint)0x9be3e0a3u, (jint)0x131da070u, 5));
  report("combine_negative", FN(nativeCombine)(&g_env, NULL, 1, 2, -1));

  /* a gather list: "123" (pos 0, lim 3), "xx456" (pos 2, lim 5), "789yy" (pos 0, lim 3) */
  static uint8_t s1[] = "123", s2[] = "xx456", s3[] = "789yy";
  struct _jobject g1 = arr(K_BUFFER, s1, 3), g2 = arr(K_BUFFER, s2, 5), g3 = arr(K_BUFFER, s3, 5);
  g1.pos = 0, g1.lim = 3, g2.pos = 2, g2.lim = 5, g3.pos = 0, g3.lim = 3;
  jobject list[3] = {&g1, &g2, &g3};
  struct _jobject lst = arr(K_OBJS, list, 3);
  report("direct_all", FN(nativeUpdateDirectAll)(&g_env, NULL, 0, &lst));
  g2.lim = 9; /* limit past the capacity */
  report("direct_all_bounds", FN(nativeUpdateDirectAll)(&g_env, NULL, 0, &lst));
  g2.lim = 5;
  jobject list_heap[2] = {&g1, &heap_buf};
  struct _jobject lst_heap = arr(K_OBJS, list_heap, 2);
  report("direct_all_heap", FN(nativeUpdateDirectAll)(&g_env, NULL, 0, &lst_heap));

  /* batch entries: argument errors are raised before any device work */
  jint pos[3] = {0, 0, 0}, len[3] = {3, 3, 3}, out[3] = {0, 0, 0}, short_out[2] = {0, 0};
  struct _jobject jpos = arr(K_INTS, pos, 3), jlen = arr(K_INTS, len, 3), jout = arr(K_INTS, out, 3);
  struct _jobject jshort = arr(K_INTS, short_out, 2);
  FN(nativeBatchDirect)(&g_env, NULL, &lst, &jpos, &jlen, NULL, &jshort, 0);
  report("batch_short_out", 0);
  FN(nativeBatchDirect)(&g_env, NULL, &lst, &jpos, NULL, NULL, &jout, 0);
  report("batch_null", 0);
  len[1] = 6; /* buffer 2 holds 5 bytes */
  FN(nativeBatchDirect)(&g_env, NULL, &lst, &jpos, &jlen, NULL, &jout, 0);
  report("batch_bounds", 0);

  jlong offs[2] = {0, 4};
  jint st[2] = {0, 0}, st_short[1] = {0};
  struct _jobject joffs = arr(K_LONGS, offs, 2), jst = arr(K_INTS, st, 2), jst1 = arr(K_INTS, st_short, 1);
  FN(nativeVerifyMessages)(&g_env, NULL, &direct_buf, &joffs, &jst1, NULL, 0);
  report("verify_short_status", 0);
  FN(nativeVerifyMessages)(&g_env, NULL, &heap_buf, &joffs, &jst, NULL, 0);
  report("verify_heap", 0);
  FN(nativeVerifyMessages)(&g_env, NULL, NULL, &joffs, &jst, NULL, 0);
  report("verify_null", 0);

  /* batched transform: argument errors first, then (no context for device 0 here) the device error */
  jlong xo[2] = {0, 4}, xol[2] = {0, 0}, xol1[1] = {0};
  int16_t xlife1[1] = {0};
  jint xst[2] = {0, 0};
  static uint8_t xout[64];
  struct _jobject jxo = arr(K_LONGS, xo, 2), jxol = arr(K_LONGS, xol, 2), jxol1 = arr(K_LONGS, xol1, 1);
  struct _jobject jxlife1 = arr(K_SHORTS, xlife1, 1), jxst = arr(K_INTS, xst, 2), xdst = arr(K_BUFFER, xout, 64);
  FN(nativeTransformMessages)(&g_env, NULL, &direct_buf, &jxo, NULL, 3, &xdst, NULL, &jxol1, &jxst, 0);
  report("xform_short_lens", 0);
  FN(nativeTransformMessages)(&g_env, NULL, &direct_buf, &jxo, &jxlife1, 3, &xdst, NULL, &jxol, &jxst, 0);
  report("xform_short_life", 0);
  FN(nativeTransformMessages)(&g_env, NULL, &direct_buf, &jxo, NULL, 3, NULL, NULL, &jxol, &jxst, 0);
  report("xform_null_out", 0);
  FN(nativeTransformMessages)(&g_env, NULL, &heap_buf, &jxo, NULL, 3, &xdst, NULL, &jxol, &jxst, 0);
  report("xform_heap", 0);
  FN(nativeTransformMessages)(&g_env, NULL, &direct_buf, &jxo, NULL, 3, &xdst, NULL, &jxol, &jxst, 0);
  report("xform_no_context", 0);

  /* chain: argument errors (the message hop itself: test_jni_recovery_chain_cpu) */
  jlong co[2] = {0, 0};
  struct _jobject jco = arr(K_LONGS, co, 2);
  report("chain_null", FN(nativeChainMessages)(&g_env, NULL, NULL, 0, &jco));
  report("chain_heap", FN(nativeChainMessages)(&g_env, NULL, &heap_buf, 0, &jco));
  report("chain_negative", FN(nativeChainMessages)(&g_env, NULL, &direct_buf, -1, &jco));
  report("chain_none", FN(nativeChainMessages)(&g_env, NULL, &direct_buf, 0, &jco)); /* "123456789": no header */

  /* host-resident dispatch policy: argument errors, and no context (no GPU initialised yet) */
  jdouble rates[3] = {0, 0, 0};
  struct _jobject jrates = arr(K_DOUBLES, rates, 3), jrates2 = arr(K_DOUBLES, rates, 2);
  report("policy_no_context", FN(nativeSetHostPolicy)(&g_env, NULL, 0, 1));
  report("rates_null", FN(nativeHostRates)(&g_env, NULL, 0, NULL));
  report("rates_short", FN(nativeHostRates)(&g_env, NULL, 0, &jrates2));
  report("rates_no_context", FN(nativeHostRates)(&g_env, NULL, 0, &jrates));
  report("last_path_no_context", FN(nativeLastHostPath)(&g_env, NULL, 0));
  report("cpu_threads_set", FN(nativeSetHostCpuThreads)(&g_env, NULL, -1, 3));
  report("cpu_threads_prev", FN(nativeSetHostCpuThreads)(&g_env, NULL, -1, 0));
  report("cpu_threads_bad", FN(nativeSetHostCpuThreads)(&g_env, NULL, -1, -1));
  report("cpu_threads_no_context", FN(nativeSetHostCpuThreads)(&g_env, NULL, 0, 2));

  FN(nativeInit)(&g_env, NULL, 0); /* no GPU in the build container: the init error is thrown */
  report("init_no_gpu", 0);
  return 0;
}
