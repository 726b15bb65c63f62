/*
 * khst_jni.c — the JNI binding of libkhst.so's host-buffer entry points (include/khst.h) for
 * khipu's JVM side, class khipu.trie.gpu.Khst (INTEGRATION.md §3 has the Scala declarations).
 *
 *   cc -std=c99 -shared -fPIC -I$JAVA_HOME/include -I$JAVA_HOME/include/linux -Iinclude \
 *      jni/khst_jni.c -Lkhipu_amd -lkhst -o libkhst_jni.so
 *
 * tests/test_jni_shim.py compiles it against include/khst.h (with a declaration-only jni.h,
 * the image has no JDK) and links it against libkhst.so with --no-undefined, and checks that
 * every host entry point of khst.h has a wrapper here.
 *
 * Conventions:
 *   - no JNI critical region is ever held: a library call may wait for the context's mutex
 *     while another thread's commit runs and then run milliseconds to seconds of GPU work,
 *     and a JVM thread inside GetPrimitiveArrayCritical must not block (HotSpot's GC locker
 *     would stall every allocating thread for that time).  byte[] / int[] / long[] inputs are
 *     copied out with Get<Type>ArrayRegion into malloc'd buffers (one memcpy: ~0.3 ms for a
 *     configs[2] block's ~3 MB) and outputs copied back with Set<Type>ArrayRegion — only the
 *     part the call wrote;
 *   - the large fresh builds (a state root over 100M accounts: ~10 GB of inputs) also take
 *     direct ByteBuffers (the *Direct wrappers): GetDirectBufferAddress, no copy, no pinning by
 *     the JVM; the library stages them over PCIe in pinned chunks, keys first, while the build
 *     runs (khst.h "host inputs");
 *   - a failing call throws: KH_EINVAL -> MerklePatriciaTrie.MPTException; KH_ENODE ->
 *     MerklePatriciaTrie.MPTNodeMissingException(message, hash, storage)
 *     (MerklePatriciaTrie.scala:46-47), built by the Scala factory Khst.nodeMissing(String,
 *     byte[]) that knows the handle's node storage (the case class has no (String)
 *     constructor, and Ledger.scala:511/542 match on its hash and storage); anything else ->
 *     khipu.trie.gpu.DeviceException; the message is kh_last_error();
 *   - KH_ENOSPC (an output array too small) does not throw: the wrapper returns a negative
 *     count or fills the `sizes` array, and the Scala side grows its arrays and calls again;
 *   - resident handles (kh_trie*) are jlongs; free() takes the long[1] the handle lives in and
 *     zeroes it, so a second free (or a finalizer after close) is a no-op, never a double free.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <jni.h>

#include "khst.h"

#define CLS "khipu/trie/gpu/Khst"

/* the class to throw; a missing class leaves its NoClassDefFoundError pending */
static void throw_cls(JNIEnv* env, const char* name, const char* msg) {
  jclass c = (*env)->FindClass(env, name);
  if (c) (*env)->ThrowNew(env, c, msg);
}

/* MPTNodeMissingException for the missing node's hash (32 bytes; zeros if unknown) */
static void throw_node_missing(JNIEnv* env, const uint8_t* hash32) {
  static const uint8_t zero[32] = {0};
  const char* msg = kh_last_error();
  jclass k = (*env)->FindClass(env, CLS);
  if (!k) return;
  jmethodID f = (*env)->GetStaticMethodID(env, k, "nodeMissing", "(Ljava/lang/String;[B)Ljava/lang/Throwable;");
  if (!f) return; /* NoSuchMethodError pending */
  jstring s = (*env)->NewStringUTF(env, msg);
  jbyteArray h = (*env)->NewByteArray(env, 32);
  if (!s || !h) return; /* OutOfMemoryError pending */
  (*env)->SetByteArrayRegion(env, h, 0, 32, (const jbyte*)(hash32 ? hash32 : zero));
  jthrowable t = (jthrowable)(*env)->CallStaticObjectMethod(env, k, f, s, h);
  if ((*env)->ExceptionCheck(env)) return; /* the factory threw: that exception stands */
  if (t) {
    (*env)->Throw(env, t);
    return;
  }
  throw_cls(env, "khipu/trie/gpu/DeviceException", msg);
}

static void throw_kh_hash(JNIEnv* env, int rc, const uint8_t* missing32) {
  if (rc == KH_ENODE) {
    throw_node_missing(env, missing32);
    return;
  }
  if (rc == KH_ENOMEM) {
    throw_cls(env, "java/lang/OutOfMemoryError", kh_last_error());
    return;
  }
  throw_cls(env, rc == KH_EINVAL ? "khipu/trie/MerklePatriciaTrie$MPTException" : "khipu/trie/gpu/DeviceException",
            kh_last_error());
}
static void throw_kh(JNIEnv* env, int rc) { throw_kh_hash(env, rc, NULL); }

/* ---- host copies of Java arrays (no critical regions) ----
 * A Bufs holds every buffer one wrapper call allocates; bufs_free releases them all.  An input
 * copy of a NULL array is NULL; of an empty one a valid 1-byte allocation.  On allocation
 * failure `oom` is set and the wrapper throws OutOfMemoryError without calling the library. */
typedef struct {
  void* p[24];
  int n;
  int oom;
} Bufs;
static void* bufs_alloc(Bufs* b, size_t bytes) {
  if (b->oom || b->n == 24) {
    b->oom = 1;
    return NULL;
  }
  void* p = malloc(bytes ? bytes : 1);
  if (!p) {
    b->oom = 1;
    return NULL;
  }
  b->p[b->n++] = p;
  return p;
}
static void bufs_free(Bufs* b) {
  for (int i = 0; i < b->n; ++i) free(b->p[i]);
  b->n = 0;
}
/* true (and OutOfMemoryError thrown) when an allocation failed */
static int bufs_failed(JNIEnv* env, Bufs* b) {
  if (!b->oom) return 0;
  bufs_free(b);
  throw_cls(env, "java/lang/OutOfMemoryError", "khst_jni: host copy of the arguments");
  return 1;
}
static jsize len_of(JNIEnv* env, jarray a) { return a ? (*env)->GetArrayLength(env, a) : 0; }
static const uint8_t* in_b(JNIEnv* env, Bufs* b, jbyteArray a) {
  if (!a) return NULL;
  const jsize n = len_of(env, a);
  jbyte* p = bufs_alloc(b, (size_t)n);
  if (p && n) (*env)->GetByteArrayRegion(env, a, 0, n, p);
  return (const uint8_t*)p;
}
static const uint32_t* in_i(JNIEnv* env, Bufs* b, jintArray a) {
  if (!a) return NULL;
  const jsize n = len_of(env, a);
  jint* p = bufs_alloc(b, 4 * (size_t)n);
  if (p && n) (*env)->GetIntArrayRegion(env, a, 0, n, p);
  return (const uint32_t*)p;
}
static const uint64_t* in_l(JNIEnv* env, Bufs* b, jlongArray a) {
  if (!a) return NULL;
  const jsize n = len_of(env, a);
  jlong* p = bufs_alloc(b, 8 * (size_t)n);
  if (p && n) (*env)->GetLongArrayRegion(env, a, 0, n, p);
  return (const uint64_t*)p;
}
/* an output buffer the size of array a (NULL array: NULL) */
static void* out_buf(JNIEnv* env, Bufs* b, jarray a, size_t esz) {
  return a ? bufs_alloc(b, esz * (size_t)len_of(env, a)) : NULL;
}
/* copy the first n elements of an output buffer back (clamped to the array) */
static void put_b(JNIEnv* env, jbyteArray a, const void* p, uint64_t n) {
  const jsize L = len_of(env, a);
  if (a && p && n) (*env)->SetByteArrayRegion(env, a, 0, n < (uint64_t)L ? (jsize)n : L, (const jbyte*)p);
}
static void put_i(JNIEnv* env, jintArray a, const void* p, uint64_t n) {
  const jsize L = len_of(env, a);
  if (a && p && n) (*env)->SetIntArrayRegion(env, a, 0, n < (uint64_t)L ? (jsize)n : L, (const jint*)p);
}
static void put_l(JNIEnv* env, jlongArray a, const void* p, uint64_t n) {
  const jsize L = len_of(env, a);
  if (a && p && n) (*env)->SetLongArrayRegion(env, a, 0, n < (uint64_t)L ? (jsize)n : L, (const jlong*)p);
}

/* entries of an offsets array (n + 1 offsets -> n items; NULL or empty -> 0) */
static uint64_t count_of(JNIEnv* env, jlongArray off) {
  const jsize n = len_of(env, off);
  return n > 0 ? (uint64_t)(n - 1) : 0;
}
static jbyteArray bytes_of(JNIEnv* env, const uint8_t* p, jsize n) {
  jbyteArray out = (*env)->NewByteArray(env, n);
  if (out) (*env)->SetByteArrayRegion(env, out, 0, n, (const jbyte*)p);
  return out;
}
static kh_trie* H(jlong h) { return (kh_trie*)(intptr_t)h; }
/* kh_stats -> long[] statsOut (nullable): n_inputs, n_leaves, n_branches, n_extensions, n_inline,
 * n_node_hashes, n_node_perms, n_key_perms, arena_bytes, n_levels, full_sort */
static void put_stats(JNIEnv* env, jlongArray out, const kh_stats* s) {
  if (!out) return;
  const jlong v[11] = {(jlong)s->n_inputs,      (jlong)s->n_leaves,     (jlong)s->n_branches, (jlong)s->n_extensions,
                       (jlong)s->n_inline,      (jlong)s->n_node_hashes, (jlong)s->n_node_perms,
                       (jlong)s->n_key_perms,   (jlong)s->arena_bytes,  (jlong)s->n_levels,   (jlong)s->full_sort};
  put_l(env, out, v, 11);
}

/* ---- direct ByteBuffers (the *Direct wrappers): the address, or NULL with an
 * IllegalArgumentException pending when the buffer is not direct or holds fewer than `need`
 * bytes (a NULL buffer is allowed when need == 0) */
static void* direct(JNIEnv* env, jobject buf, uint64_t need, const char* what) {
  if (!buf) {
    if (need) throw_cls(env, "java/lang/IllegalArgumentException", what);
    return NULL;
  }
  void* p = (*env)->GetDirectBufferAddress(env, buf);
  const jlong cap = (*env)->GetDirectBufferCapacity(env, buf);
  if (!p || cap < 0 || (uint64_t)cap < need) {
    throw_cls(env, "java/lang/IllegalArgumentException", what);
    return NULL;
  }
  return p;
}
/* the keys / value offsets / values of n inputs in direct buffers, capacities checked */
typedef struct {
  const uint8_t* keys;
  const uint64_t* voff;
  const uint8_t* vals;
} DirectIn;
static int direct_inputs(JNIEnv* env, jobject keys, jint klen, jobject vals, jobject voff, jlong n, DirectIn* in) {
  if (n < 0 || klen < 0) {
    throw_cls(env, "java/lang/IllegalArgumentException", "negative count or key length");
    return 0;
  }
  in->keys = direct(env, keys, (uint64_t)n * (uint64_t)klen, "keys: not a direct buffer of n * klen bytes");
  if ((*env)->ExceptionCheck(env)) return 0;
  in->voff = direct(env, voff, 8 * ((uint64_t)n + 1), "voff: not a direct buffer of n + 1 longs (native order)");
  if ((*env)->ExceptionCheck(env)) return 0;
  const uint64_t vend = n ? in->voff[n] : 0;
  if (n && in->voff[n] < in->voff[0]) {
    throw_cls(env, "java/lang/IllegalArgumentException", "voff: not monotone");
    return 0;
  }
  in->vals = direct(env, vals, vend, "vals: not a direct buffer of voff[n] bytes");
  return !(*env)->ExceptionCheck(env);
}

/* ---- library ---- */
JNIEXPORT jbyteArray JNICALL Java_khipu_trie_gpu_Khst_version(JNIEnv* env, jclass cls) {
  (void)cls;
  const char* v = kh_version();
  return bytes_of(env, (const uint8_t*)v, (jsize)strlen(v));
}
JNIEXPORT jint JNICALL Java_khipu_trie_gpu_Khst_deviceCount(JNIEnv* env, jclass cls) {
  (void)env, (void)cls;
  return kh_device_count();
}

/* ---- crypto.kec256 over a batch (crypto/package.scala:37-47): messages data[off[i]..off[i+1]) */
JNIEXPORT jbyteArray JNICALL Java_khipu_trie_gpu_Khst_kec256Batch(JNIEnv* env, jclass cls, jbyteArray data,
                                                                 jlongArray off) {
  (void)cls;
  const uint64_t n = count_of(env, off);
  Bufs b = {0};
  const uint8_t* d = in_b(env, &b, data);
  const uint64_t* o = in_l(env, &b, off);
  uint8_t* r = bufs_alloc(&b, 32 * (size_t)n);
  if (bufs_failed(env, &b)) return NULL;
  const int rc = kh_kec256_batch(d, o, n, r);
  jbyteArray out = rc == KH_OK ? bytes_of(env, r, (jsize)(32 * n)) : NULL;
  bufs_free(&b);
  if (rc != KH_OK) throw_kh(env, rc);
  return out;
}

/* ---- fresh tries (TrieAccounts.flush / TrieStorage.flush / GenesisDataLoader) ---- */
/* keys: n*klen bytes, vals packed with voff (n+1 offsets); returns the root */
JNIEXPORT jbyteArray JNICALL Java_khipu_trie_gpu_Khst_trieRoot(JNIEnv* env, jclass cls, jbyteArray keys, jint klen,
                                                              jbyteArray vals, jlongArray voff, jint flags,
                                                              jlongArray statsOut) {
  (void)cls;
  const uint64_t n = count_of(env, voff);
  uint8_t root[32];
  kh_stats st;
  Bufs b = {0};
  const uint8_t* k = in_b(env, &b, keys);
  const uint8_t* v = in_b(env, &b, vals);
  const uint64_t* o = in_l(env, &b, voff);
  if (bufs_failed(env, &b)) return NULL;
  const int rc = kh_trie_root(k, (uint32_t)klen, v, o, n, (uint32_t)flags, root, &st);
  bufs_free(&b);
  if (rc != KH_OK) {
    throw_kh(env, rc);
    return NULL;
  }
  put_stats(env, statsOut, &st);
  return bytes_of(env, root, 32);
}

/* the same over direct buffers (keys: n*klen bytes, voff: n+1 native-order longs, vals:
 * voff[n] bytes): no copy on the JVM side; the library stages the inputs over PCIe while the
 * build runs */
JNIEXPORT jbyteArray JNICALL Java_khipu_trie_gpu_Khst_trieRootDirect(JNIEnv* env, jclass cls, jobject keys, jint klen,
                                                                    jobject vals, jobject voff, jlong n, jint flags,
                                                                    jlongArray statsOut) {
  (void)cls;
  DirectIn in;
  if (!direct_inputs(env, keys, klen, vals, voff, n, &in)) return NULL;
  uint8_t root[32];
  kh_stats st;
  const int rc = kh_trie_root(in.keys, (uint32_t)klen, in.vals, in.voff, (uint64_t)n, (uint32_t)flags, root, &st);
  if (rc != KH_OK) {
    throw_kh(env, rc);
    return NULL;
  }
  put_stats(env, statsOut, &st);
  return bytes_of(env, root, 32);
}

/* nseg tries (segOff: nseg+1 input offsets); returns nseg*32 bytes of roots */
JNIEXPORT jbyteArray JNICALL Java_khipu_trie_gpu_Khst_trieRootsSegmented(JNIEnv* env, jclass cls, jbyteArray keys,
                                                                        jint klen, jbyteArray vals, jlongArray voff,
                                                                        jlongArray segOff, jint flags) {
  (void)cls;
  const uint64_t nseg = count_of(env, segOff);
  Bufs b = {0};
  const uint8_t* k = in_b(env, &b, keys);
  const uint8_t* v = in_b(env, &b, vals);
  const uint64_t* o = in_l(env, &b, voff);
  const uint64_t* so = in_l(env, &b, segOff);
  uint8_t* r = bufs_alloc(&b, 32 * (size_t)nseg);
  if (bufs_failed(env, &b)) return NULL;
  const int rc = kh_trie_roots_segmented(k, (uint32_t)klen, v, o, so, nseg, (uint32_t)flags, r, NULL);
  jbyteArray out = rc == KH_OK ? bytes_of(env, r, (jsize)(32 * nseg)) : NULL;
  bufs_free(&b);
  if (rc != KH_OK) throw_kh(env, rc);
  return out;
}

/* the same over the listed devices of this JVM (contiguous trie ranges, no exchange) */
JNIEXPORT jbyteArray JNICALL Java_khipu_trie_gpu_Khst_trieRootsSegmentedSharded(
    JNIEnv* env, jclass cls, jintArray devices, jbyteArray keys, jint klen, jbyteArray vals, jlongArray voff,
    jlongArray segOff, jint flags) {
  (void)cls;
  const uint64_t nseg = count_of(env, segOff);
  const jsize ng = len_of(env, devices);
  Bufs b = {0};
  const uint32_t* d = in_i(env, &b, devices);
  const uint8_t* k = in_b(env, &b, keys);
  const uint8_t* v = in_b(env, &b, vals);
  const uint64_t* o = in_l(env, &b, voff);
  const uint64_t* so = in_l(env, &b, segOff);
  uint8_t* r = bufs_alloc(&b, 32 * (size_t)nseg);
  if (bufs_failed(env, &b)) return NULL;
  const int rc =
      kh_trie_roots_segmented_sharded((const int*)d, (int)ng, k, (uint32_t)klen, v, o, so, nseg, (uint32_t)flags, r, NULL);
  jbyteArray out = rc == KH_OK ? bytes_of(env, r, (jsize)(32 * nseg)) : NULL;
  bufs_free(&b);
  if (rc != KH_OK) throw_kh(env, rc);
  return out;
}

/* variable-length unhashed keys (keys[koff[i]..koff[i+1]), 0..32 bytes); nseg tries */
JNIEXPORT jbyteArray JNICALL Java_khipu_trie_gpu_Khst_trieRootsVarkeys(JNIEnv* env, jclass cls, jbyteArray keys,
                                                                      jlongArray koff, jbyteArray vals,
                                                                      jlongArray voff, jlongArray segOff) {
  (void)cls;
  const uint64_t nseg = count_of(env, segOff);
  Bufs b = {0};
  const uint8_t* k = in_b(env, &b, keys);
  const uint64_t* ko = in_l(env, &b, koff);
  const uint8_t* v = in_b(env, &b, vals);
  const uint64_t* o = in_l(env, &b, voff);
  const uint64_t* so = in_l(env, &b, segOff);
  uint8_t* r = bufs_alloc(&b, 32 * (size_t)nseg);
  if (bufs_failed(env, &b)) return NULL;
  const int rc = kh_trie_roots_varkeys(k, ko, v, o, so, nseg, r, NULL);
  jbyteArray out = rc == KH_OK ? bytes_of(env, r, (jsize)(32 * nseg)) : NULL;
  bufs_free(&b);
  if (rc != KH_OK) throw_kh(env, rc);
  return out;
}

/* every block's transactions (or receipts) root in one call (MptListValidator.scala:15-46) */
JNIEXPORT jbyteArray JNICALL Java_khipu_trie_gpu_Khst_listRoots(JNIEnv* env, jclass cls, jbyteArray items,
                                                               jlongArray off, jlongArray segOff) {
  (void)cls;
  const uint64_t nseg = count_of(env, segOff);
  Bufs b = {0};
  const uint8_t* it = in_b(env, &b, items);
  const uint64_t* o = in_l(env, &b, off);
  const uint64_t* so = in_l(env, &b, segOff);
  uint8_t* r = bufs_alloc(&b, 32 * (size_t)nseg);
  if (bufs_failed(env, &b)) return NULL;
  const int rc = kh_list_roots(it, o, so, nseg, r, NULL);
  jbyteArray out = rc == KH_OK ? bytes_of(env, r, (jsize)(32 * nseg)) : NULL;
  bufs_free(&b);
  if (rc != KH_OK) throw_kh(env, rc);
  return out;
}

/* the root on several GPUs of this JVM (nibble shards, RCCL point-to-point exchange) */
JNIEXPORT jbyteArray JNICALL Java_khipu_trie_gpu_Khst_trieRootSharded(JNIEnv* env, jclass cls, jintArray devices,
                                                                     jbyteArray keys, jint klen, jbyteArray vals,
                                                                     jlongArray voff, jint flags) {
  (void)cls;
  const uint64_t n = count_of(env, voff);
  const jsize ng = len_of(env, devices);
  uint8_t root[32];
  Bufs b = {0};
  const uint32_t* d = in_i(env, &b, devices);
  const uint8_t* k = in_b(env, &b, keys);
  const uint8_t* v = in_b(env, &b, vals);
  const uint64_t* o = in_l(env, &b, voff);
  if (bufs_failed(env, &b)) return NULL;
  const int rc = kh_trie_root_sharded((const int*)d, (int)ng, k, (uint32_t)klen, v, o, n, (uint32_t)flags, root, NULL);
  bufs_free(&b);
  if (rc != KH_OK) {
    throw_kh(env, rc);
    return NULL;
  }
  return bytes_of(env, root, 32);
}

/* the same over direct buffers (as trieRootDirect) */
JNIEXPORT jbyteArray JNICALL Java_khipu_trie_gpu_Khst_trieRootShardedDirect(JNIEnv* env, jclass cls, jintArray devices,
                                                                           jobject keys, jint klen, jobject vals,
                                                                           jobject voff, jlong n, jint flags) {
  (void)cls;
  DirectIn in;
  if (!direct_inputs(env, keys, klen, vals, voff, n, &in)) return NULL;
  const jsize ng = len_of(env, devices);
  uint8_t root[32];
  Bufs b = {0};
  const uint32_t* d = in_i(env, &b, devices);
  if (bufs_failed(env, &b)) return NULL;
  const int rc = kh_trie_root_sharded((const int*)d, (int)ng, in.keys, (uint32_t)klen, in.vals, in.voff, (uint64_t)n,
                                      (uint32_t)flags, root, NULL);
  bufs_free(&b);
  if (rc != KH_OK) {
    throw_kh(env, rc);
    return NULL;
  }
  return bytes_of(env, root, 32);
}

/* Root + the node set a fresh store needs (GenesisDataLoader.scala:139-147, persist of a fresh
 * trie): the caller's hashes (32 per node), rlp and off (n_nodes + 1) arrays receive the nodes;
 * sizes[0] / sizes[1] = nodes / RLP bytes.  Returns the root, or NULL when an output array is
 * too small (sizes then hold what is needed: grow and call again). */
JNIEXPORT jbyteArray JNICALL Java_khipu_trie_gpu_Khst_trieRootNodes(JNIEnv* env, jclass cls, jbyteArray keys,
                                                                   jint klen, jbyteArray vals, jlongArray voff,
                                                                   jint flags, jbyteArray hashes, jbyteArray rlp,
                                                                   jlongArray off, jlongArray sizes) {
  (void)cls;
  const uint64_t n = count_of(env, voff);
  const uint64_t node_cap = (uint64_t)len_of(env, hashes) / 32, rlp_cap = (uint64_t)len_of(env, rlp);
  const jsize noff = len_of(env, off);
  const uint64_t cap = node_cap < (uint64_t)(noff > 0 ? noff - 1 : 0) ? node_cap : (uint64_t)(noff > 0 ? noff - 1 : 0);
  uint8_t root[32];
  uint64_t nn = 0, nb = 0;
  Bufs b = {0};
  const uint8_t* k = in_b(env, &b, keys);
  const uint8_t* v = in_b(env, &b, vals);
  const uint64_t* o = in_l(env, &b, voff);
  uint8_t* hs = out_buf(env, &b, hashes, 1);
  uint8_t* rl = out_buf(env, &b, rlp, 1);
  uint64_t* of = out_buf(env, &b, off, 8);
  if (bufs_failed(env, &b)) return NULL;
  const int rc = kh_trie_root_nodes(k, (uint32_t)klen, v, o, n, (uint32_t)flags, root, hs, cap, rl, rlp_cap, of, &nn,
                                    &nb, NULL);
  if (rc == KH_OK) {
    put_b(env, hashes, hs, 32 * nn);
    put_b(env, rlp, rl, nb);
    put_l(env, off, of, nn + 1);
  }
  bufs_free(&b);
  const jlong sz[2] = {(jlong)nn, (jlong)nb};
  put_l(env, sizes, sz, 2);
  if (rc == KH_ENOSPC) return NULL;
  if (rc != KH_OK) {
    throw_kh(env, rc);
    return NULL;
  }
  return bytes_of(env, root, 32);
}

/* the same over direct buffers: inputs as trieRootDirect; outputs hashes (32 per node), rlp and
 * off (n_nodes + 1 native-order longs) are direct buffers too, written in place (a 100M-account
 * state's node set is ~20 GB: no Java array holds it) */
JNIEXPORT jbyteArray JNICALL Java_khipu_trie_gpu_Khst_trieRootNodesDirect(JNIEnv* env, jclass cls, jobject keys,
                                                                         jint klen, jobject vals, jobject voff, jlong n,
                                                                         jint flags, jobject hashes, jobject rlp,
                                                                         jobject off, jlongArray sizes) {
  (void)cls;
  DirectIn in;
  if (!direct_inputs(env, keys, klen, vals, voff, n, &in)) return NULL;
  uint8_t* hs = direct(env, hashes, 0, "hashes: not a direct buffer");
  uint8_t* rl = (*env)->ExceptionCheck(env) ? NULL : direct(env, rlp, 0, "rlp: not a direct buffer");
  uint64_t* of = (*env)->ExceptionCheck(env) ? NULL : direct(env, off, 0, "off: not a direct buffer");
  if ((*env)->ExceptionCheck(env)) return NULL;
  const jlong hcap = hashes ? (*env)->GetDirectBufferCapacity(env, hashes) : 0;
  const jlong rcap = rlp ? (*env)->GetDirectBufferCapacity(env, rlp) : 0;
  const jlong ocap = off ? (*env)->GetDirectBufferCapacity(env, off) : 0;
  const uint64_t node_cap = (uint64_t)hcap / 32, ocount = ocap >= 8 ? (uint64_t)ocap / 8 - 1 : 0;
  const uint64_t cap = node_cap < ocount ? node_cap : ocount;
  uint8_t root[32];
  uint64_t nn = 0, nb = 0;
  const int rc = kh_trie_root_nodes(in.keys, (uint32_t)klen, in.vals, in.voff, (uint64_t)n, (uint32_t)flags, root, hs,
                                    cap, rl, (uint64_t)rcap, of, &nn, &nb, NULL);
  const jlong sz[2] = {(jlong)nn, (jlong)nb};
  put_l(env, sizes, sz, 2);
  if (rc == KH_ENOSPC) return NULL;
  if (rc != KH_OK) {
    throw_kh(env, rc);
    return NULL;
  }
  return bytes_of(env, root, 32);
}

/* ---- fast sync: NodeDatasRequest.processResponse (sync/package.scala:81-165) ---- */
/* per value: hash32 (32 each), match (-1: none), status; nchild (per value) and the children
 * 16 slots per value (child32: 512 bytes, childKind: 16 per value) */
JNIEXPORT void JNICALL Java_khipu_trie_gpu_Khst_verifyNodes(JNIEnv* env, jclass cls, jbyteArray data, jlongArray off,
                                                           jbyteArray req32, jbyteArray reqKind, jbyteArray hash32,
                                                           jlongArray match, jbyteArray status, jbyteArray nchild,
                                                           jbyteArray child32, jbyteArray childKind) {
  (void)cls;
  const uint64_t n = count_of(env, off), nreq = (uint64_t)len_of(env, reqKind);
  Bufs b = {0};
  const uint8_t* dt = in_b(env, &b, data);
  const uint64_t* o = in_l(env, &b, off);
  const uint8_t* rq = in_b(env, &b, req32);
  const uint8_t* rk = in_b(env, &b, reqKind);
  uint8_t* hs = out_buf(env, &b, hash32, 1);
  int64_t* mt = out_buf(env, &b, match, 8);
  uint8_t* stt = out_buf(env, &b, status, 1);
  uint8_t* nc = out_buf(env, &b, nchild, 1);
  uint8_t* c32 = out_buf(env, &b, child32, 1);
  uint8_t* ck = out_buf(env, &b, childKind, 1);
  if (bufs_failed(env, &b)) return;
  const int rc = kh_verify_nodes(dt, o, n, rq, rk, nreq, hs, mt, stt, nc, c32, ck);
  if (rc == KH_OK) {
    put_b(env, hash32, hs, 32 * n);
    put_l(env, match, mt, n);
    put_b(env, status, stt, n);
    put_b(env, nchild, nc, n);
    put_b(env, child32, c32, 512 * n);
    put_b(env, childKind, ck, 16 * n);
  }
  bufs_free(&b);
  if (rc != KH_OK) throw_kh(env, rc);
}

/* the same with the children packed as processResponse concatenates them (childOff: n+1);
 * returns the number of children, or its negation when child32 / childKind are too small
 * (every other output is written: grow and call again) */
JNIEXPORT jlong JNICALL Java_khipu_trie_gpu_Khst_verifyNodesPacked(JNIEnv* env, jclass cls, jbyteArray data,
                                                                  jlongArray off, jbyteArray req32, jbyteArray reqKind,
                                                                  jlongArray match, jbyteArray status,
                                                                  jlongArray childOff, jbyteArray child32,
                                                                  jbyteArray childKind) {
  (void)cls;
  const uint64_t n = count_of(env, off), nreq = (uint64_t)len_of(env, reqKind);
  const uint64_t cap = (uint64_t)len_of(env, childKind);
  uint64_t nch = 0;
  Bufs b = {0};
  const uint8_t* dt = in_b(env, &b, data);
  const uint64_t* o = in_l(env, &b, off);
  const uint8_t* rq = in_b(env, &b, req32);
  const uint8_t* rk = in_b(env, &b, reqKind);
  uint8_t* hashes = bufs_alloc(&b, 32 * (size_t)n);
  int64_t* mt = out_buf(env, &b, match, 8);
  uint8_t* stt = out_buf(env, &b, status, 1);
  uint64_t* co = out_buf(env, &b, childOff, 8);
  uint8_t* c32 = out_buf(env, &b, child32, 1);
  uint8_t* ck = out_buf(env, &b, childKind, 1);
  if (bufs_failed(env, &b)) return 0;
  const int rc = kh_verify_nodes_packed(dt, o, n, rq, rk, nreq, hashes, mt, stt, co, c32, ck, cap, &nch);
  if (rc == KH_OK || rc == KH_ENOSPC) {
    put_l(env, match, mt, n);
    put_b(env, status, stt, n);
    put_l(env, childOff, co, n + 1);
  }
  if (rc == KH_OK) {
    put_b(env, child32, c32, 32 * nch);
    put_b(env, childKind, ck, nch);
  }
  bufs_free(&b);
  if (rc == KH_ENOSPC) return -(jlong)nch;
  if (rc != KH_OK) {
    throw_kh(env, rc);
    return 0;
  }
  return (jlong)nch;
}

/* ---- resident tries (BlockWorldState / TrieAccounts / TrieStorage over a live state) ---- */
/* open from records (flags: HASH_KEYS, EMIT_NODES); rootOut (byte[32], nullable) gets the root */
JNIEXPORT jlong JNICALL Java_khipu_trie_gpu_Khst_openHost(JNIEnv* env, jclass cls, jbyteArray keys, jint klen,
                                                         jbyteArray vals, jlongArray voff, jint flags,
                                                         jbyteArray rootOut) {
  (void)cls;
  const uint64_t n = count_of(env, voff);
  uint8_t root[32];
  kh_trie* h = NULL;
  Bufs b = {0};
  const uint8_t* k = in_b(env, &b, keys);
  const uint8_t* v = in_b(env, &b, vals);
  const uint64_t* o = in_l(env, &b, voff);
  if (bufs_failed(env, &b)) return 0;
  const int rc = kh_trie_open_host(k, (uint32_t)klen, v, o, n, (uint32_t)flags, root, &h);
  bufs_free(&b);
  if (rc != KH_OK) {
    throw_kh(env, rc);
    return 0;
  }
  put_b(env, rootOut, root, 32);
  return (jlong)(intptr_t)h;
}

/* the same over direct buffers (as trieRootDirect): a 50M-account state opened without a copy */
JNIEXPORT jlong JNICALL Java_khipu_trie_gpu_Khst_openHostDirect(JNIEnv* env, jclass cls, jobject keys, jint klen,
                                                               jobject vals, jobject voff, jlong n, jint flags,
                                                               jbyteArray rootOut) {
  (void)cls;
  DirectIn in;
  if (!direct_inputs(env, keys, klen, vals, voff, n, &in)) return 0;
  uint8_t root[32];
  kh_trie* h = NULL;
  const int rc = kh_trie_open_host(in.keys, (uint32_t)klen, in.vals, in.voff, (uint64_t)n, (uint32_t)flags, root, &h);
  if (rc != KH_OK) {
    throw_kh(env, rc);
    return 0;
  }
  put_b(env, rootOut, root, 32);
  return (jlong)(intptr_t)h;
}

/* MerklePatriciaTrie.apply(rootHash, source) (MerklePatriciaTrie.scala:60-66): open from a node
 * store (encodings enc[off[i]..off[i+1]), content addressed); a missing node throws
 * MPTNodeMissingException (with its hash) after writing the hash into missingOut (byte[32],
 * nullable) */
JNIEXPORT jlong JNICALL Java_khipu_trie_gpu_Khst_openNodes(JNIEnv* env, jclass cls, jbyteArray root32,
                                                          jbyteArray enc, jlongArray off, jint flags,
                                                          jbyteArray missingOut) {
  (void)cls;
  const uint64_t n = count_of(env, off);
  uint8_t missing[32] = {0};
  kh_trie* h = NULL;
  Bufs b = {0};
  const uint8_t* r = in_b(env, &b, root32);
  const uint8_t* e = in_b(env, &b, enc);
  const uint64_t* o = in_l(env, &b, off);
  if (bufs_failed(env, &b)) return 0;
  if (!r || len_of(env, root32) < 32) {
    bufs_free(&b);
    throw_cls(env, "java/lang/IllegalArgumentException", "root32: 32 bytes");
    return 0;
  }
  const int rc = kh_trie_open_nodes_host(r, e, o, n, (uint32_t)flags, missing, &h);
  bufs_free(&b);
  if (rc == KH_ENODE) put_b(env, missingOut, missing, 32);
  if (rc != KH_OK) {
    throw_kh_hash(env, rc, missing);
    return 0;
  }
  return (jlong)(intptr_t)h;
}

/* one commit (upserts then deletes) on a single trie; returns the new root */
JNIEXPORT jbyteArray JNICALL Java_khipu_trie_gpu_Khst_apply(JNIEnv* env, jclass cls, jlong handle, jbyteArray upKeys,
                                                           jbyteArray upVals, jlongArray upVoff, jbyteArray delKeys,
                                                           jint klen, jint flags, jlongArray statsOut) {
  (void)cls;
  const uint64_t nup = count_of(env, upVoff), ndel = klen > 0 ? (uint64_t)(len_of(env, delKeys) / klen) : 0;
  uint8_t root[32];
  kh_stats st;
  Bufs b = {0};
  const uint8_t* k = in_b(env, &b, upKeys);
  const uint8_t* v = in_b(env, &b, upVals);
  const uint64_t* o = in_l(env, &b, upVoff);
  const uint8_t* d = in_b(env, &b, delKeys);
  if (bufs_failed(env, &b)) return NULL;
  const int rc = kh_trie_apply_host(H(handle), k, v, o, nup, d, ndel, (uint32_t)klen, (uint32_t)flags, root, &st);
  bufs_free(&b);
  if (rc != KH_OK) {
    throw_kh(env, rc);
    return NULL;
  }
  put_stats(env, statsOut, &st);
  return bytes_of(env, root, 32);
}

/* a forest of tries (contract storage) on the host entry points' context */
JNIEXPORT jlong JNICALL Java_khipu_trie_gpu_Khst_forestOpen(JNIEnv* env, jclass cls, jint flags) {
  (void)cls;
  kh_trie* h = NULL;
  const int rc = kh_forest_open(NULL, (uint32_t)flags, &h);
  if (rc != KH_OK) {
    throw_kh(env, rc);
    return 0;
  }
  return (jlong)(intptr_t)h;
}

/* one commit of many tries' ops (each op names its trie); triesOut / rootsOut receive the
 * touched tries and their new roots; returns their number (negated: the outputs were short) */
JNIEXPORT jlong JNICALL Java_khipu_trie_gpu_Khst_forestApply(JNIEnv* env, jclass cls, jlong handle, jintArray upTrie,
                                                            jbyteArray upKeys, jbyteArray upVals, jlongArray upVoff,
                                                            jintArray delTrie, jbyteArray delKeys, jint klen,
                                                            jintArray triesOut, jbyteArray rootsOut) {
  (void)cls;
  const uint64_t nup = count_of(env, upVoff), ndel = (uint64_t)len_of(env, delTrie);
  const jsize tcap = len_of(env, triesOut), rcap = len_of(env, rootsOut) / 32;
  const uint64_t cap = (uint64_t)(tcap < rcap ? tcap : rcap);
  uint64_t nt = 0;
  Bufs b = {0};
  const uint32_t* ut = in_i(env, &b, upTrie);
  const uint8_t* k = in_b(env, &b, upKeys);
  const uint8_t* v = in_b(env, &b, upVals);
  const uint64_t* o = in_l(env, &b, upVoff);
  const uint32_t* dt = in_i(env, &b, delTrie);
  const uint8_t* d = in_b(env, &b, delKeys);
  uint32_t* to = out_buf(env, &b, triesOut, 4);
  uint8_t* ro = out_buf(env, &b, rootsOut, 1);
  if (bufs_failed(env, &b)) return 0;
  const int rc = kh_forest_apply_host(H(handle), ut, k, v, o, nup, dt, d, ndel, (uint32_t)klen, to, ro, cap, &nt, NULL);
  if (rc == KH_OK) {
    put_i(env, triesOut, to, nt);
    put_b(env, rootsOut, ro, 32 * nt);
  }
  bufs_free(&b);
  if (rc == KH_ENOSPC) return -(jlong)nt; /* committed; kh_forest_last_roots reads them again */
  if (rc != KH_OK) {
    throw_kh(env, rc);
    return 0;
  }
  return (jlong)nt;
}

/* the last commit's touched tries and roots (after a short forestApply, or a rollback) */
JNIEXPORT jlong JNICALL Java_khipu_trie_gpu_Khst_forestLastRoots(JNIEnv* env, jclass cls, jlong handle,
                                                                jintArray triesOut, jbyteArray rootsOut) {
  (void)cls;
  const jsize tcap = len_of(env, triesOut), rcap = len_of(env, rootsOut) / 32;
  const uint64_t cap = (uint64_t)(tcap < rcap ? tcap : rcap);
  uint64_t nt = 0;
  Bufs b = {0};
  uint32_t* to = out_buf(env, &b, triesOut, 4);
  uint8_t* ro = out_buf(env, &b, rootsOut, 1);
  if (bufs_failed(env, &b)) return 0;
  const int rc = kh_forest_last_roots(H(handle), to, ro, cap, &nt);
  if (rc == KH_OK) {
    put_i(env, triesOut, to, nt);
    put_b(env, rootsOut, ro, 32 * nt);
  }
  bufs_free(&b);
  if (rc == KH_ENOSPC) return -(jlong)nt;
  if (rc != KH_OK) {
    throw_kh(env, rc);
    return 0;
  }
  return (jlong)nt;
}

/* One block (BlockWorldState.scala:243-252 then TrieAccounts.flush): storage ops into the
 * forest, the new storage roots written into the named account bodies (accTrie[i], -1 =
 * KH_NO_TRIE: none), the account ops into the state trie.  All or nothing.  Returns the state
 * root. */
JNIEXPORT jbyteArray JNICALL Java_khipu_trie_gpu_Khst_blockCommit(
    JNIEnv* env, jclass cls, jlong state, jlong storage, jintArray slotTrie, jbyteArray slotKeys, jbyteArray slotVals,
    jlongArray slotVoff, jintArray delSlotTrie, jbyteArray delSlotKeys, jint slotKlen, jbyteArray accKeys,
    jbyteArray accBodies, jlongArray accVoff, jintArray accTrie, jbyteArray delAccKeys, jint accKlen,
    jlongArray statsOut) {
  (void)cls;
  const uint64_t ns_up = count_of(env, slotVoff), ns_del = (uint64_t)len_of(env, delSlotTrie);
  const uint64_t na_up = count_of(env, accVoff);
  const uint64_t na_del = accKlen > 0 ? (uint64_t)(len_of(env, delAccKeys) / accKlen) : 0;
  uint8_t root[32];
  kh_stats st;
  Bufs b = {0};
  const uint32_t* st_ = in_i(env, &b, slotTrie);
  const uint8_t* sk = in_b(env, &b, slotKeys);
  const uint8_t* sv = in_b(env, &b, slotVals);
  const uint64_t* so = in_l(env, &b, slotVoff);
  const uint32_t* sdt = in_i(env, &b, delSlotTrie);
  const uint8_t* sdk = in_b(env, &b, delSlotKeys);
  const uint8_t* ak = in_b(env, &b, accKeys);
  const uint8_t* av = in_b(env, &b, accBodies);
  const uint64_t* ao = in_l(env, &b, accVoff);
  const uint32_t* at = in_i(env, &b, accTrie);
  const uint8_t* adk = in_b(env, &b, delAccKeys);
  if (bufs_failed(env, &b)) return NULL;
  const int rc = kh_block_commit_host(H(state), H(storage), st_, sk, sv, so, ns_up, sdt, sdk, ns_del,
                                      (uint32_t)slotKlen, ak, av, ao, at, na_up, adk, na_del, (uint32_t)accKlen, root,
                                      &st);
  bufs_free(&b);
  if (rc != KH_OK) {
    throw_kh(env, rc);
    return NULL;
  }
  put_stats(env, statsOut, &st);
  return bytes_of(env, root, 32);
}

/* BlockWorldState.persist (BlockWorldState.scala:312-330): the nodes the last commit created
 * (opened with EMIT_NODES) into hashes / rlp / off; sizes[0] / sizes[1] = nodes / RLP bytes.
 * Returns the node count, or -1 when an output array is too small (sizes hold what is
 * needed: grow and call again; nothing is re-encoded). */
JNIEXPORT jlong JNICALL Java_khipu_trie_gpu_Khst_emitNodes(JNIEnv* env, jclass cls, jlong handle, jbyteArray hashes,
                                                          jbyteArray rlp, jlongArray off, jlongArray sizes) {
  (void)cls;
  const uint64_t node_cap = (uint64_t)len_of(env, hashes) / 32, rlp_cap = (uint64_t)len_of(env, rlp);
  const jsize noff = len_of(env, off);
  const uint64_t cap = node_cap < (uint64_t)(noff > 0 ? noff - 1 : 0) ? node_cap : (uint64_t)(noff > 0 ? noff - 1 : 0);
  uint64_t nn = 0, nb = 0;
  Bufs b = {0};
  uint8_t* hs = out_buf(env, &b, hashes, 1);
  uint8_t* rl = out_buf(env, &b, rlp, 1);
  uint64_t* of = out_buf(env, &b, off, 8);
  if (bufs_failed(env, &b)) return 0;
  const int rc = kh_trie_emit_nodes(H(handle), hs, cap, rl, rlp_cap, of, &nn, &nb);
  if (rc == KH_OK) {
    put_b(env, hashes, hs, 32 * nn);
    put_b(env, rlp, rl, nb);
    put_l(env, off, of, nn + 1);
  }
  bufs_free(&b);
  const jlong sz[2] = {(jlong)nn, (jlong)nb};
  put_l(env, sizes, sz, 2);
  if (rc == KH_ENOSPC) return -1;
  if (rc != KH_OK) {
    throw_kh(env, rc);
    return 0;
  }
  return (jlong)nn;
}

/* MerklePatriciaTrie.get for a batch (MerklePatriciaTrie.scala:90-147): byte[][] with null for
 * an absent key (None); trieIds (int[], nullable) for a forest.  The value bytes' size is
 * negotiated: a call that finds them larger than the buffer returns KH_ENOSPC with the size;
 * another thread's commit on the handle between two calls can change it again, so the loop
 * grows and retries (bounded) as khipu_amd/device.py does. */
#define GET_TRIES 16
JNIEXPORT jobjectArray JNICALL Java_khipu_trie_gpu_Khst_get(JNIEnv* env, jclass cls, jlong handle, jintArray trieIds,
                                                           jbyteArray keys, jint klen) {
  (void)cls;
  const jsize n = klen > 0 ? len_of(env, keys) / klen : 0;
  Bufs b = {0};
  const uint32_t* t = in_i(env, &b, trieIds);
  const uint8_t* k = in_b(env, &b, keys);
  uint8_t* found = bufs_alloc(&b, (size_t)n);
  uint64_t* voff = bufs_alloc(&b, 8 * ((size_t)n + 1));
  if (bufs_failed(env, &b)) return NULL;
  uint64_t need = 0, cap = 0;
  uint8_t* vals = NULL;
  int rc = KH_ENOSPC;
  for (int tries = 0; rc == KH_ENOSPC && tries < GET_TRIES; ++tries) { /* the first call reports the bytes needed */
    rc = kh_trie_get_host(H(handle), t, k, (uint32_t)klen, (uint64_t)n, vals, cap, voff, found, &need);
    if (rc == KH_ENOSPC) {
      free(vals);
      cap = need + need / 8; /* headroom for a concurrent commit that grows the values again */
      vals = malloc((size_t)(cap ? cap : 1));
      if (!vals) rc = KH_ENOMEM;
    }
  }
  jobjectArray out = NULL;
  if (rc == KH_OK) {
    jclass ba = (*env)->FindClass(env, "[B");
    out = ba ? (*env)->NewObjectArray(env, n, ba, NULL) : NULL;
    for (jsize i = 0; out && i < n; ++i) {
      if (!found[i]) continue; /* None */
      jbyteArray v = bytes_of(env, vals + voff[i], (jsize)(voff[i + 1] - voff[i]));
      if (!v) break; /* OutOfMemoryError pending */
      (*env)->SetObjectArrayElement(env, out, i, v);
      (*env)->DeleteLocalRef(env, v);
    }
  }
  free(vals);
  bufs_free(&b);
  if (rc != KH_OK) throw_kh(env, rc);
  return out;
}

/* ---- versions (Ledger.scala:237-271 retry / reject; TrieAccounts.rootHash; copy) ---- */
JNIEXPORT jint JNICALL Java_khipu_trie_gpu_Khst_savepoint(JNIEnv* env, jclass cls, jlong handle) {
  (void)cls;
  uint32_t depth = 0;
  const int rc = kh_trie_savepoint(H(handle), &depth);
  if (rc != KH_OK) throw_kh(env, rc);
  return (jint)depth;
}
JNIEXPORT void JNICALL Java_khipu_trie_gpu_Khst_rollback(JNIEnv* env, jclass cls, jlong handle) {
  (void)cls;
  const int rc = kh_trie_rollback(H(handle));
  if (rc != KH_OK) throw_kh(env, rc);
}
JNIEXPORT void JNICALL Java_khipu_trie_gpu_Khst_release(JNIEnv* env, jclass cls, jlong handle) {
  (void)cls;
  const int rc = kh_trie_release(H(handle));
  if (rc != KH_OK) throw_kh(env, rc);
}
JNIEXPORT jint JNICALL Java_khipu_trie_gpu_Khst_savepointDepth(JNIEnv* env, jclass cls, jlong handle) {
  (void)cls;
  uint32_t depth = 0;
  const int rc = kh_trie_savepoint_depth(H(handle), &depth);
  if (rc != KH_OK) throw_kh(env, rc);
  return (jint)depth;
}

/* TrieAccounts.rootHash of pending logs (TrieAccounts.scala:73-80): the root the batch would
 * give, the handle unchanged */
JNIEXPORT jbyteArray JNICALL Java_khipu_trie_gpu_Khst_rootOf(JNIEnv* env, jclass cls, jlong handle, jbyteArray upKeys,
                                                            jbyteArray upVals, jlongArray upVoff, jbyteArray delKeys,
                                                            jint klen, jint flags) {
  (void)cls;
  const uint64_t nup = count_of(env, upVoff), ndel = klen > 0 ? (uint64_t)(len_of(env, delKeys) / klen) : 0;
  uint8_t root[32];
  Bufs b = {0};
  const uint8_t* k = in_b(env, &b, upKeys);
  const uint8_t* v = in_b(env, &b, upVals);
  const uint64_t* o = in_l(env, &b, upVoff);
  const uint8_t* d = in_b(env, &b, delKeys);
  if (bufs_failed(env, &b)) return NULL;
  const int rc = kh_trie_root_of_host(H(handle), k, v, o, nup, d, ndel, (uint32_t)klen, (uint32_t)flags, root, NULL);
  bufs_free(&b);
  if (rc != KH_OK) {
    throw_kh(env, rc);
    return NULL;
  }
  return bytes_of(env, root, 32);
}

/* MerklePatriciaTrie.copy (MerklePatriciaTrie.scala:556): a new handle (free it with free) */
JNIEXPORT jlong JNICALL Java_khipu_trie_gpu_Khst_copy(JNIEnv* env, jclass cls, jlong handle) {
  (void)cls;
  kh_trie* out = NULL;
  const int rc = kh_trie_copy(H(handle), &out);
  if (rc != KH_OK) {
    throw_kh(env, rc);
    return 0;
  }
  return (jlong)(intptr_t)out;
}

/* ---- memory of a resident handle ---- */
/* usageOut (long[6]): records, live records, heap bytes, live heap bytes, map slots, HBM bytes */
JNIEXPORT void JNICALL Java_khipu_trie_gpu_Khst_usage(JNIEnv* env, jclass cls, jlong handle, jlongArray usageOut) {
  (void)cls;
  kh_trie_usage_t u;
  const int rc = kh_trie_usage(H(handle), &u);
  if (rc != KH_OK) {
    throw_kh(env, rc);
    return;
  }
  const jlong v[6] = {(jlong)u.records,         (jlong)u.live_records, (jlong)u.heap_bytes,
                      (jlong)u.live_heap_bytes, (jlong)u.map_slots,    (jlong)u.hbm_bytes};
  put_l(env, usageOut, v, 6);
}
/* rewrite the live records densely between blocks (no savepoint open); beforeOut (long[2],
 * nullable): records / heap bytes before */
JNIEXPORT void JNICALL Java_khipu_trie_gpu_Khst_compact(JNIEnv* env, jclass cls, jlong handle, jlongArray beforeOut) {
  (void)cls;
  kh_trie_usage_t u;
  const int rc = kh_trie_compact(H(handle), &u);
  if (rc != KH_OK) {
    throw_kh(env, rc);
    return;
  }
  const jlong v[2] = {(jlong)u.records, (jlong)u.heap_bytes};
  put_l(env, beforeOut, v, 2);
}
JNIEXPORT jlong JNICALL Java_khipu_trie_gpu_Khst_size(JNIEnv* env, jclass cls, jlong handle) {
  (void)cls;
  uint64_t n = 0;
  const int rc = kh_trie_size(H(handle), &n);
  if (rc != KH_OK) throw_kh(env, rc);
  return (jlong)n;
}
/* Free the handle held in handleBox[0] and zero it there: idempotent (the library cannot guard
 * a raw pointer, so the box is what makes a second close or a finalizer harmless).  The
 * wrapper is not itself reentrant for one box: the Scala owner closes from one thread. */
JNIEXPORT void JNICALL Java_khipu_trie_gpu_Khst_free(JNIEnv* env, jclass cls, jlongArray handleBox) {
  (void)cls;
  if (!handleBox || len_of(env, handleBox) < 1) return;
  jlong h = 0;
  (*env)->GetLongArrayRegion(env, handleBox, 0, 1, &h);
  if (!h) return;
  const jlong zero = 0;
  (*env)->SetLongArrayRegion(env, handleBox, 0, 1, &zero); /* zeroed before the free: never freed twice */
  const int rc = kh_trie_free(H(h));
  if (rc != KH_OK) throw_kh(env, rc);
}
