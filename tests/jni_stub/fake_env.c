/* TEST INFRASTRUCTURE ONLY: a minimal in-process JNIEnv for tests/jni_stub/jni.h, so the shim's
 * wrappers (jni/khst_jni.c) run without a JVM.  Objects are FakeObj records: arrays (heap
 * copies), direct buffers (address + capacity), classes, strings and throwables.  It records
 * the pending exception (class and message) and the calls of the Scala factory
 * Khst.nodeMissing(String, byte[]) the shim uses for MPTNodeMissingException.
 *
 * jni_driver (tests/jni_stub/jni_driver.c) drives the wrappers through it; test_jni_shim.py and
 * test_gpu_jni.py run the driver. */
#include <stdarg.h>
#include <stdlib.h>
#include <string.h>

#include "fake_env.h"

static FakeObj* obj_new(int kind) {
  FakeObj* o = calloc(1, sizeof(FakeObj));
  o->kind = kind;
  return o;
}
FakeObj* fake_array(jsize len, int esz, const void* init) {
  FakeObj* o = obj_new(FK_ARRAY);
  o->len = len;
  o->esz = esz;
  o->data = calloc((size_t)len * esz + 1, 1);
  if (init) memcpy(o->data, init, (size_t)len * esz);
  return o;
}
FakeObj* fake_direct(void* p, jlong cap) {
  FakeObj* o = obj_new(FK_DIRECT);
  o->data = p;
  o->cap = cap;
  return o;
}

FakeState fake;

static jclass FindClass(JNIEnv* env, const char* name) {
  (void)env;
  FakeObj* o = obj_new(FK_CLASS);
  strncpy(o->name, name, sizeof(o->name) - 1);
  return (jclass)o;
}
static void set_pending(const char* cls, const char* msg) {
  fake.pending = 1;
  strncpy(fake.exc_class, cls, sizeof(fake.exc_class) - 1);
  strncpy(fake.exc_msg, msg ? msg : "", sizeof(fake.exc_msg) - 1);
}
static jint ThrowNew(JNIEnv* env, jclass clazz, const char* msg) {
  (void)env;
  set_pending(((FakeObj*)clazz)->name, msg);
  return 0;
}
static void DeleteLocalRef(JNIEnv* env, jobject obj) { (void)env, (void)obj; }
static jsize GetArrayLength(JNIEnv* env, jarray a) {
  (void)env;
  return ((FakeObj*)a)->len;
}
static jobjectArray NewObjectArray(JNIEnv* env, jsize len, jclass clazz, jobject init) {
  (void)env, (void)clazz, (void)init;
  return (jobjectArray)fake_array(len, (int)sizeof(void*), NULL);
}
static void SetObjectArrayElement(JNIEnv* env, jobjectArray a, jsize i, jobject v) {
  (void)env;
  ((FakeObj**)((FakeObj*)a)->data)[i] = (FakeObj*)v;
}
static jbyteArray NewByteArray(JNIEnv* env, jsize len) {
  (void)env;
  return (jbyteArray)fake_array(len, 1, NULL);
}
static void region(FakeObj* o, jsize start, jsize len, void* buf, int get) {
  if (start < 0 || len < 0 || start + len > o->len) {
    set_pending("java/lang/ArrayIndexOutOfBoundsException", "region");
    return;
  }
  char* p = (char*)o->data + (size_t)start * o->esz;
  if (get)
    memcpy(buf, p, (size_t)len * o->esz);
  else
    memcpy(p, buf, (size_t)len * o->esz);
  fake.region_bytes += (uint64_t)len * o->esz;
}
static void GetLongArrayRegion(JNIEnv* env, jlongArray a, jsize s, jsize n, jlong* b) { (void)env, region((FakeObj*)a, s, n, b, 1); }
static void GetIntArrayRegion(JNIEnv* env, jintArray a, jsize s, jsize n, jint* b) { (void)env, region((FakeObj*)a, s, n, b, 1); }
static void GetByteArrayRegion(JNIEnv* env, jbyteArray a, jsize s, jsize n, jbyte* b) { (void)env, region((FakeObj*)a, s, n, b, 1); }
static void SetByteArrayRegion(JNIEnv* env, jbyteArray a, jsize s, jsize n, const jbyte* b) {
  (void)env, region((FakeObj*)a, s, n, (void*)b, 0);
}
static void SetLongArrayRegion(JNIEnv* env, jlongArray a, jsize s, jsize n, const jlong* b) {
  (void)env, region((FakeObj*)a, s, n, (void*)b, 0);
}
static void SetIntArrayRegion(JNIEnv* env, jintArray a, jsize s, jsize n, const jint* b) {
  (void)env, region((FakeObj*)a, s, n, (void*)b, 0);
}
static void* GetDirectBufferAddress(JNIEnv* env, jobject b) {
  (void)env;
  return ((FakeObj*)b)->kind == FK_DIRECT ? ((FakeObj*)b)->data : NULL;
}
static jlong GetDirectBufferCapacity(JNIEnv* env, jobject b) {
  (void)env;
  return ((FakeObj*)b)->kind == FK_DIRECT ? ((FakeObj*)b)->cap : -1;
}
static struct _jmethodID* const NODE_MISSING = (struct _jmethodID*)0x1;
static jmethodID GetStaticMethodID(JNIEnv* env, jclass c, const char* name, const char* sig) {
  (void)env;
  if (!strcmp(((FakeObj*)c)->name, "khipu/trie/gpu/Khst") && !strcmp(name, "nodeMissing") &&
      !strcmp(sig, "(Ljava/lang/String;[B)Ljava/lang/Throwable;"))
    return NODE_MISSING;
  set_pending("java/lang/NoSuchMethodError", name);
  return NULL;
}
static jobject CallStaticObjectMethod(JNIEnv* env, jclass c, jmethodID m, ...) {
  (void)env, (void)c;
  if (m != NODE_MISSING) return NULL;
  va_list ap;
  va_start(ap, m);
  FakeObj* s = va_arg(ap, FakeObj*);
  FakeObj* h = va_arg(ap, FakeObj*);
  va_end(ap);
  fake.node_missing_calls++;
  memcpy(fake.node_missing_hash, h->data, 32);
  FakeObj* t = obj_new(FK_THROWABLE);
  strcpy(t->name, "khipu/trie/MerklePatriciaTrie$MPTNodeMissingException");
  strncpy(t->msg, s->msg, sizeof(t->msg) - 1);
  return (jobject)t;
}
static jint Throw(JNIEnv* env, jthrowable t) {
  (void)env;
  set_pending(((FakeObj*)t)->name, ((FakeObj*)t)->msg);
  return 0;
}
static jboolean ExceptionCheck(JNIEnv* env) {
  (void)env;
  return (jboolean)fake.pending;
}
static jstring NewStringUTF(JNIEnv* env, const char* utf) {
  (void)env;
  FakeObj* o = obj_new(FK_STRING);
  strncpy(o->msg, utf, sizeof(o->msg) - 1);
  return (jstring)o;
}

static const struct JNINativeInterface_ table = {
    .FindClass = FindClass,
    .ThrowNew = ThrowNew,
    .DeleteLocalRef = DeleteLocalRef,
    .GetArrayLength = GetArrayLength,
    .NewObjectArray = NewObjectArray,
    .SetObjectArrayElement = SetObjectArrayElement,
    .NewByteArray = NewByteArray,
    .GetLongArrayRegion = GetLongArrayRegion,
    .SetByteArrayRegion = SetByteArrayRegion,
    .SetLongArrayRegion = SetLongArrayRegion,
    .SetIntArrayRegion = SetIntArrayRegion,
    .GetByteArrayRegion = GetByteArrayRegion,
    .GetIntArrayRegion = GetIntArrayRegion,
    .GetDirectBufferAddress = GetDirectBufferAddress,
    .GetDirectBufferCapacity = GetDirectBufferCapacity,
    .GetStaticMethodID = GetStaticMethodID,
    .CallStaticObjectMethod = CallStaticObjectMethod,
    .Throw = Throw,
    .ExceptionCheck = ExceptionCheck,
    .NewStringUTF = NewStringUTF,
};
static JNIEnv the_env = &table;
JNIEnv* fake_env(void) {
  memset(&fake, 0, sizeof(fake));
  return &the_env;
}
