/*
 * Test fixture, not a JDK header: the part of the JNI interface (Java Native Interface
 * Specification, "JNI Types and Data Structures" and "JNI Functions") that
 * ambry_amd/jni/ambrycrc_jni.c calls, so the shim compiles and runs against the fake JVM in
 * tests/native/jni_harness.c where no JDK is installed. Types and function signatures follow the
 * specification; the function table holds only the entries the shim uses, by name, so it is NOT
 * binary compatible with a real JNINativeInterface_ and must never be used to build the shim
 * that a JVM loads (`make -C ambry_amd jni JAVA_HOME=...` uses the JDK's jni.h).
 */
#ifndef AMBRYCRC_TEST_JNI_STUB_H
#define AMBRYCRC_TEST_JNI_STUB_H
#include <stdarg.h>
#include <stdint.h>

#define JNIEXPORT __attribute__((visibility("default")))
#define JNICALL
#define JNI_FALSE 0
#define JNI_TRUE 1
#define JNI_ABORT 2

typedef int32_t jint;
typedef int64_t jlong;
typedef int8_t jbyte;
typedef int16_t jshort;
typedef double jdouble;
typedef uint8_t jboolean;
typedef jint jsize;

struct _jobject;
typedef struct _jobject* jobject;
typedef jobject jclass;
typedef jobject jarray;
typedef jarray jbyteArray;
typedef jarray jintArray;
typedef jarray jlongArray;
typedef jarray jshortArray;
typedef jarray jdoubleArray;
typedef jarray jobjectArray;
typedef jobject jthrowable;
struct _jmethodID;
typedef struct _jmethodID* jmethodID;

struct JNINativeInterface_;
typedef const struct JNINativeInterface_* JNIEnv;

struct JNINativeInterface_ {
  jclass (*FindClass)(JNIEnv* env, const char* name);
  jint (*ThrowNew)(JNIEnv* env, jclass clazz, const char* msg);
  jboolean (*ExceptionCheck)(JNIEnv* env);
  void (*DeleteLocalRef)(JNIEnv* env, jobject obj);
  jmethodID (*GetMethodID)(JNIEnv* env, jclass clazz, const char* name, const char* sig);
  jint (*CallIntMethod)(JNIEnv* env, jobject obj, jmethodID methodID, ...);
  jsize (*GetArrayLength)(JNIEnv* env, jarray array);
  jobject (*GetObjectArrayElement)(JNIEnv* env, jobjectArray array, jsize index);
  void (*GetIntArrayRegion)(JNIEnv* env, jintArray array, jsize start, jsize len, jint* buf);
  void (*SetIntArrayRegion)(JNIEnv* env, jintArray array, jsize start, jsize len, const jint* buf);
  void (*GetLongArrayRegion)(JNIEnv* env, jlongArray array, jsize start, jsize len, jlong* buf);
  void (*SetLongArrayRegion)(JNIEnv* env, jlongArray array, jsize start, jsize len, const jlong* buf);
  void (*GetShortArrayRegion)(JNIEnv* env, jshortArray array, jsize start, jsize len, jshort* buf);
  void* (*GetPrimitiveArrayCritical)(JNIEnv* env, jarray array, jboolean* isCopy);
  void (*ReleasePrimitiveArrayCritical)(JNIEnv* env, jarray array, void* carray, jint mode);
  void* (*GetDirectBufferAddress)(JNIEnv* env, jobject buf);
  jlong (*GetDirectBufferCapacity)(JNIEnv* env, jobject buf);
  void (*SetDoubleArrayRegion)(JNIEnv* env, jdoubleArray array, jsize start, jsize len, const jdouble* buf);
};

#endif
