/* TEST INFRASTRUCTURE ONLY: a declaration-only stand-in for the JDK's jni.h (this image has
 * no JDK), holding exactly the types and JNIEnv functions jni/khst_jni.c uses, with the
 * JDK's names and signatures (jni.h of JDK 8).  tests/test_jni_shim.py compiles the shim
 * against it and include/khst.h, so a changed khst.h signature breaks the build.  The
 * function-table layout is not the JDK's: the object built here is never loaded by a JVM. */
#ifndef KHST_TEST_JNI_STUB_H
#define KHST_TEST_JNI_STUB_H
#include <stdint.h>

#define JNIEXPORT __attribute__((visibility("default")))
#define JNICALL
#define JNI_ABORT 2
#define JNI_FALSE 0
#define JNI_TRUE 1

typedef int32_t jint;
typedef int64_t jlong;
typedef int8_t jbyte;
typedef uint8_t jboolean;
typedef jint jsize;

struct _jobject;
typedef struct _jobject* jobject;
typedef jobject jclass;
typedef jobject jthrowable;
typedef jobject jarray;
typedef jarray jbyteArray;
typedef jarray jintArray;
typedef jarray jlongArray;
typedef jarray jobjectArray;
typedef jobject jstring;
struct _jmethodID;
typedef struct _jmethodID* jmethodID;

struct JNINativeInterface_;
typedef const struct JNINativeInterface_* JNIEnv;

struct JNINativeInterface_ {
  jclass (*FindClass)(JNIEnv* env, const char* name);
  jint (*ThrowNew)(JNIEnv* env, jclass clazz, const char* msg);
  void (*DeleteLocalRef)(JNIEnv* env, jobject obj);
  jsize (*GetArrayLength)(JNIEnv* env, jarray array);
  jobjectArray (*NewObjectArray)(JNIEnv* env, jsize len, jclass clazz, jobject init);
  void (*SetObjectArrayElement)(JNIEnv* env, jobjectArray array, jsize index, jobject val);
  jbyteArray (*NewByteArray)(JNIEnv* env, jsize len);
  void (*GetLongArrayRegion)(JNIEnv* env, jlongArray array, jsize start, jsize len, jlong* buf);
  void (*SetByteArrayRegion)(JNIEnv* env, jbyteArray array, jsize start, jsize len, const jbyte* buf);
  void (*SetLongArrayRegion)(JNIEnv* env, jlongArray array, jsize start, jsize len, const jlong* buf);
  void (*SetIntArrayRegion)(JNIEnv* env, jintArray array, jsize start, jsize len, const jint* buf);
  void (*GetByteArrayRegion)(JNIEnv* env, jbyteArray array, jsize start, jsize len, jbyte* buf);
  void (*GetIntArrayRegion)(JNIEnv* env, jintArray array, jsize start, jsize len, jint* buf);
  void* (*GetDirectBufferAddress)(JNIEnv* env, jobject buf);
  jlong (*GetDirectBufferCapacity)(JNIEnv* env, jobject buf);
  jmethodID (*GetStaticMethodID)(JNIEnv* env, jclass clazz, const char* name, const char* sig);
  jobject (*CallStaticObjectMethod)(JNIEnv* env, jclass clazz, jmethodID methodID, ...);
  jint (*Throw)(JNIEnv* env, jthrowable obj);
  jboolean (*ExceptionCheck)(JNIEnv* env);
  jstring (*NewStringUTF)(JNIEnv* env, const char* utf);
};

#endif
