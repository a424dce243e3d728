/* Compile-check harness for jni/sparkbam_jni.c only: the subset of the JNI types and the
 * JNIEnv function table that the shim uses, with JNI's C signatures.  NOT the JDK's jni.h
 * (member order does not follow the real table, so nothing built against it may run); the
 * shim is built for real by jni/Makefile against $JAVA_HOME/include/jni.h. */
#ifndef SBH_TEST_JNI_H
#define SBH_TEST_JNI_H
#include <stdint.h>
typedef int32_t jint;
typedef int64_t jlong;
typedef int8_t jbyte;
typedef unsigned char jboolean;
typedef jint jsize;
typedef struct _jobject *jobject;
typedef jobject jclass, jarray, jlongArray, jintArray, jobjectArray, jstring, jthrowable;
typedef struct _jmethodID *jmethodID;
#define JNIEXPORT __attribute__((visibility("default")))
#define JNICALL
#define JNI_ABORT 2
struct JNINativeInterface_;
typedef const struct JNINativeInterface_ *JNIEnv;
struct JNINativeInterface_ {
  jclass (*FindClass)(JNIEnv *, const char *);
  jint (*ThrowNew)(JNIEnv *, jclass, const char *);
  void *(*GetDirectBufferAddress)(JNIEnv *, jobject);
  jlong (*GetDirectBufferCapacity)(JNIEnv *, jobject);
  jobject (*NewDirectByteBuffer)(JNIEnv *, void *, jlong);
  jsize (*GetArrayLength)(JNIEnv *, jarray);
  void (*SetLongArrayRegion)(JNIEnv *, jlongArray, jsize, jsize, const jlong *);
  void (*GetLongArrayRegion)(JNIEnv *, jlongArray, jsize, jsize, jlong *);
  jint *(*GetIntArrayElements)(JNIEnv *, jintArray, unsigned char *);
  void (*ReleaseIntArrayElements)(JNIEnv *, jintArray, jint *, jint);
  jobject (*GetObjectArrayElement)(JNIEnv *, jobjectArray, jsize);
  jmethodID (*GetMethodID)(JNIEnv *, jclass, const char *, const char *);
  jobject (*NewObject)(JNIEnv *, jclass, jmethodID, ...);
  jint (*Throw)(JNIEnv *, jthrowable);
  jstring (*NewStringUTF)(JNIEnv *, const char *);
  jlongArray (*NewLongArray)(JNIEnv *, jsize);
  const char *(*GetStringUTFChars)(JNIEnv *, jstring, jboolean *);
  void (*ReleaseStringUTFChars)(JNIEnv *, jstring, const char *);
  void (*GetIntArrayRegion)(JNIEnv *, jintArray, jsize, jsize, jint *);
};
#endif
