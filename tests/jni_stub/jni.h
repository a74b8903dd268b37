/* Minimal stand-in for the JDK's <jni.h>, ONLY for tests/test_abi.py to compile-check
 * jni/mfhip_jni.c against include/mfhip.h in an image without a JDK.  It declares the handful of
 * JNI types and JNIEnv functions the shim uses, with the JNI specification's C signatures.  It is
 * not a JDK header and nothing built with it is linked or run. */
#ifndef MFHIP_TEST_JNI_STUB_H
#define MFHIP_TEST_JNI_STUB_H
#include <stddef.h>
#include <stdint.h>
typedef int32_t jint;
typedef int64_t jlong;
typedef int8_t jbyte;
typedef uint8_t jboolean;
typedef uint16_t jchar;
typedef double jdouble;
typedef jint jsize;
struct _jobject;
typedef struct _jobject* jobject;
typedef jobject jclass;
typedef jobject jstring;
typedef jobject jthrowable;
typedef jobject jarray;
typedef jarray jintArray;
typedef jarray jbyteArray;
typedef jarray jdoubleArray;
#define JNIEXPORT __attribute__((visibility("default")))
#define JNICALL
#define JNI_ABORT 2
struct JNINativeInterface_;
typedef const struct JNINativeInterface_* JNIEnv;
struct JNINativeInterface_ {
  jclass (*FindClass)(JNIEnv*, const char*);
  jint (*ThrowNew)(JNIEnv*, jclass, const char*);
  jsize (*GetArrayLength)(JNIEnv*, jarray);
  jint* (*GetIntArrayElements)(JNIEnv*, jintArray, jboolean*);
  void (*ReleaseIntArrayElements)(JNIEnv*, jintArray, jint*, jint);
  jdouble* (*GetDoubleArrayElements)(JNIEnv*, jdoubleArray, jboolean*);
  void (*ReleaseDoubleArrayElements)(JNIEnv*, jdoubleArray, jdouble*, jint);
  jbyte* (*GetByteArrayElements)(JNIEnv*, jbyteArray, jboolean*);
  void (*ReleaseByteArrayElements)(JNIEnv*, jbyteArray, jbyte*, jint);
  jbyteArray (*NewByteArray)(JNIEnv*, jsize);
  void (*GetByteArrayRegion)(JNIEnv*, jbyteArray, jsize, jsize, jbyte*);
  void (*SetByteArrayRegion)(JNIEnv*, jbyteArray, jsize, jsize, const jbyte*);
  void* (*GetPrimitiveArrayCritical)(JNIEnv*, jarray, jboolean*);
  void (*ReleasePrimitiveArrayCritical)(JNIEnv*, jarray, void*, jint);
  const char* (*GetStringUTFChars)(JNIEnv*, jstring, jboolean*);
  void (*ReleaseStringUTFChars)(JNIEnv*, jstring, const char*);
};
#endif
