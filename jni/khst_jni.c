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
 *   - byte[] / long[] / int[] arguments are pinned with GetPrimitiveArrayCritical for the
 *     duration of the call only (the library keeps no pointer after it returns); inputs are
 *     released with JNI_ABORT, outputs with 0 (copied back);
 *   - a failing call throws: KH_EINVAL -> MerklePatriciaTrie.MPTException, KH_ENODE ->
 *     MerklePatriciaTrie.MPTNodeMissingException (MerklePatriciaTrie.scala:46-47), anything else
 *     -> khipu.trie.gpu.DeviceException; the message is kh_last_error();
 *   - KH_ENOSPC (an output array too small) does not throw: the wrapper returns a negative
 *     count or fills the `sizes` array, and the Scala side grows its arrays and calls again;
 *   - resident handles (kh_trie*) are jlongs; free() takes the long[1] the handle lives in and
 *     zeroes it, so a second free (or a finalizer after close) is a no-op, never a double free.
 */
#include <stdint.h>
#include <stdlib.h>
#include <jni.h>

#include "khst.h"

#define CLS "khipu/trie/gpu/Khst"

static void throw_kh(JNIEnv* env, int rc) {
  const char* cls = rc == KH_EINVAL  ? "khipu/trie/MerklePatriciaTrie$MPTException"
                    : rc == KH_ENODE ? "khipu/trie/MerklePatriciaTrie$MPTNodeMissingException"
                                     : "khipu/trie/gpu/DeviceException";
  (*env)->ThrowNew(env, (*env)->FindClass(env, cls), kh_last_error());
}

/* pin / unpin (a NULL Java array stays a NULL pointer) */
static void* pin(JNIEnv* env, jarray a) { return a ? (*env)->GetPrimitiveArrayCritical(env, a, NULL) : NULL; }
static void unpin_in(JNIEnv* env, jarray a, void* p) {
  if (a && p) (*env)->ReleasePrimitiveArrayCritical(env, a, p, JNI_ABORT);
}
static void unpin_out(JNIEnv* env, jarray a, void* p) {
  if (a && p) (*env)->ReleasePrimitiveArrayCritical(env, a, p, 0);
}
static jsize len_of(JNIEnv* env, jarray a) { return a ? (*env)->GetArrayLength(env, a) : 0; }
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
  const jsize n = len_of(env, out);
  (*env)->SetLongArrayRegion(env, out, 0, n < 11 ? n : 11, v);
}

/* ---- library ---- */
JNIEXPORT jbyteArray JNICALL Java_khipu_trie_gpu_Khst_version(JNIEnv* env, jclass cls) {
  (void)cls;
  const char* v = kh_version();
  jsize n = 0;
  while (v[n]) ++n;
  return bytes_of(env, (const uint8_t*)v, n);
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
  jbyteArray out = (*env)->NewByteArray(env, (jsize)(32 * n));
  if (!out) return NULL;
  jbyte* d = pin(env, data);
  jlong* o = pin(env, off);
  jbyte* r = pin(env, out);
  const int rc = kh_kec256_batch((const uint8_t*)d, (const uint64_t*)o, n, (uint8_t*)r);
  unpin_out(env, out, r);
  unpin_in(env, off, o);
  unpin_in(env, data, d);
  if (rc != KH_OK) {
    throw_kh(env, rc);
    return NULL;
  }
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
  jbyte* k = pin(env, keys);
  jbyte* v = pin(env, vals);
  jlong* o = pin(env, voff);
  const int rc = kh_trie_root((const uint8_t*)k, (uint32_t)klen, (const uint8_t*)v, (const uint64_t*)o, n,
                              (uint32_t)flags, root, &st);
  unpin_in(env, voff, o);
  unpin_in(env, vals, v);
  unpin_in(env, keys, k);
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
  jbyteArray out = (*env)->NewByteArray(env, (jsize)(32 * nseg));
  if (!out) return NULL;
  jbyte* k = pin(env, keys);
  jbyte* v = pin(env, vals);
  jlong* o = pin(env, voff);
  jlong* so = pin(env, segOff);
  jbyte* r = pin(env, out);
  const int rc = kh_trie_roots_segmented((const uint8_t*)k, (uint32_t)klen, (const uint8_t*)v, (const uint64_t*)o,
                                         (const uint64_t*)so, nseg, (uint32_t)flags, (uint8_t*)r, NULL);
  unpin_out(env, out, r);
  unpin_in(env, segOff, so);
  unpin_in(env, voff, o);
  unpin_in(env, vals, v);
  unpin_in(env, keys, k);
  if (rc != KH_OK) {
    throw_kh(env, rc);
    return NULL;
  }
  return out;
}

/* the same over the listed devices of this JVM (contiguous trie ranges, no exchange) */
JNIEXPORT jbyteArray JNICALL Java_khipu_trie_gpu_Khst_trieRootsSegmentedSharded(
    JNIEnv* env, jclass cls, jintArray devices, jbyteArray keys, jint klen, jbyteArray vals, jlongArray voff,
    jlongArray segOff, jint flags) {
  (void)cls;
  const uint64_t nseg = count_of(env, segOff);
  const jsize ng = len_of(env, devices);
  jbyteArray out = (*env)->NewByteArray(env, (jsize)(32 * nseg));
  if (!out) return NULL;
  jint* d = pin(env, devices);
  jbyte* k = pin(env, keys);
  jbyte* v = pin(env, vals);
  jlong* o = pin(env, voff);
  jlong* so = pin(env, segOff);
  jbyte* r = pin(env, out);
  const int rc = kh_trie_roots_segmented_sharded((const int*)d, (int)ng, (const uint8_t*)k, (uint32_t)klen,
                                                 (const uint8_t*)v, (const uint64_t*)o, (const uint64_t*)so, nseg,
                                                 (uint32_t)flags, (uint8_t*)r, NULL);
  unpin_out(env, out, r);
  unpin_in(env, segOff, so);
  unpin_in(env, voff, o);
  unpin_in(env, vals, v);
  unpin_in(env, keys, k);
  unpin_in(env, devices, d);
  if (rc != KH_OK) {
    throw_kh(env, rc);
    return NULL;
  }
  return out;
}

/* variable-length unhashed keys (keys[koff[i]..koff[i+1]), 0..32 bytes); nseg tries */
JNIEXPORT jbyteArray JNICALL Java_khipu_trie_gpu_Khst_trieRootsVarkeys(JNIEnv* env, jclass cls, jbyteArray keys,
                                                                      jlongArray koff, jbyteArray vals,
                                                                      jlongArray voff, jlongArray segOff) {
  (void)cls;
  const uint64_t nseg = count_of(env, segOff);
  jbyteArray out = (*env)->NewByteArray(env, (jsize)(32 * nseg));
  if (!out) return NULL;
  jbyte* k = pin(env, keys);
  jlong* ko = pin(env, koff);
  jbyte* v = pin(env, vals);
  jlong* o = pin(env, voff);
  jlong* so = pin(env, segOff);
  jbyte* r = pin(env, out);
  const int rc = kh_trie_roots_varkeys((const uint8_t*)k, (const uint64_t*)ko, (const uint8_t*)v, (const uint64_t*)o,
                                       (const uint64_t*)so, nseg, (uint8_t*)r, NULL);
  unpin_out(env, out, r);
  unpin_in(env, segOff, so);
  unpin_in(env, voff, o);
  unpin_in(env, vals, v);
  unpin_in(env, koff, ko);
  unpin_in(env, keys, k);
  if (rc != KH_OK) {
    throw_kh(env, rc);
    return NULL;
  }
  return out;
}

/* every block's transactions (or receipts) root in one call (MptListValidator.scala:15-46) */
JNIEXPORT jbyteArray JNICALL Java_khipu_trie_gpu_Khst_listRoots(JNIEnv* env, jclass cls, jbyteArray items,
                                                               jlongArray off, jlongArray segOff) {
  (void)cls;
  const uint64_t nseg = count_of(env, segOff);
  jbyteArray out = (*env)->NewByteArray(env, (jsize)(32 * nseg));
  if (!out) return NULL;
  jbyte* it = pin(env, items);
  jlong* o = pin(env, off);
  jlong* so = pin(env, segOff);
  jbyte* r = pin(env, out);
  const int rc = kh_list_roots((const uint8_t*)it, (const uint64_t*)o, (const uint64_t*)so, nseg, (uint8_t*)r, NULL);
  unpin_out(env, out, r);
  unpin_in(env, segOff, so);
  unpin_in(env, off, o);
  unpin_in(env, items, it);
  if (rc != KH_OK) {
    throw_kh(env, rc);
    return NULL;
  }
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
  jint* d = pin(env, devices);
  jbyte* k = pin(env, keys);
  jbyte* v = pin(env, vals);
  jlong* o = pin(env, voff);
  const int rc = kh_trie_root_sharded((const int*)d, (int)ng, (const uint8_t*)k, (uint32_t)klen, (const uint8_t*)v,
                                      (const uint64_t*)o, n, (uint32_t)flags, root, NULL);
  unpin_in(env, voff, o);
  unpin_in(env, vals, v);
  unpin_in(env, keys, k);
  unpin_in(env, devices, d);
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
  jbyte* k = pin(env, keys);
  jbyte* v = pin(env, vals);
  jlong* o = pin(env, voff);
  jbyte* hs = pin(env, hashes);
  jbyte* rl = pin(env, rlp);
  jlong* of = pin(env, off);
  const int rc = kh_trie_root_nodes((const uint8_t*)k, (uint32_t)klen, (const uint8_t*)v, (const uint64_t*)o, n,
                                    (uint32_t)flags, root, (uint8_t*)hs, cap, (uint8_t*)rl, rlp_cap, (uint64_t*)of,
                                    &nn, &nb, NULL);
  unpin_out(env, off, of);
  unpin_out(env, rlp, rl);
  unpin_out(env, hashes, hs);
  unpin_in(env, voff, o);
  unpin_in(env, vals, v);
  unpin_in(env, keys, k);
  const jlong sz[2] = {(jlong)nn, (jlong)nb};
  if (sizes) (*env)->SetLongArrayRegion(env, sizes, 0, len_of(env, sizes) < 2 ? len_of(env, sizes) : 2, sz);
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
  jbyte* dt = pin(env, data);
  jlong* o = pin(env, off);
  jbyte* rq = pin(env, req32);
  jbyte* rk = pin(env, reqKind);
  jbyte* hs = pin(env, hash32);
  jlong* mt = pin(env, match);
  jbyte* stt = pin(env, status);
  jbyte* nc = pin(env, nchild);
  jbyte* c32 = pin(env, child32);
  jbyte* ck = pin(env, childKind);
  const int rc = kh_verify_nodes((const uint8_t*)dt, (const uint64_t*)o, n, (const uint8_t*)rq, (const uint8_t*)rk,
                                 nreq, (uint8_t*)hs, (int64_t*)mt, (uint8_t*)stt, (uint8_t*)nc, (uint8_t*)c32,
                                 (uint8_t*)ck);
  unpin_out(env, childKind, ck);
  unpin_out(env, child32, c32);
  unpin_out(env, nchild, nc);
  unpin_out(env, status, stt);
  unpin_out(env, match, mt);
  unpin_out(env, hash32, hs);
  unpin_in(env, reqKind, rk);
  unpin_in(env, req32, rq);
  unpin_in(env, off, o);
  unpin_in(env, data, dt);
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
  uint8_t* hashes = malloc(32 * (size_t)(n ? n : 1));
  if (!hashes) {
    (*env)->ThrowNew(env, (*env)->FindClass(env, "java/lang/OutOfMemoryError"), "verifyNodesPacked");
    return 0;
  }
  uint64_t nch = 0;
  jbyte* dt = pin(env, data);
  jlong* o = pin(env, off);
  jbyte* rq = pin(env, req32);
  jbyte* rk = pin(env, reqKind);
  jlong* mt = pin(env, match);
  jbyte* stt = pin(env, status);
  jlong* co = pin(env, childOff);
  jbyte* c32 = pin(env, child32);
  jbyte* ck = pin(env, childKind);
  const int rc = kh_verify_nodes_packed((const uint8_t*)dt, (const uint64_t*)o, n, (const uint8_t*)rq,
                                        (const uint8_t*)rk, nreq, hashes, (int64_t*)mt, (uint8_t*)stt, (uint64_t*)co,
                                        (uint8_t*)c32, (uint8_t*)ck, cap, &nch);
  unpin_out(env, childKind, ck);
  unpin_out(env, child32, c32);
  unpin_out(env, childOff, co);
  unpin_out(env, status, stt);
  unpin_out(env, match, mt);
  unpin_in(env, reqKind, rk);
  unpin_in(env, req32, rq);
  unpin_in(env, off, o);
  unpin_in(env, data, dt);
  free(hashes);
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
  jbyte* k = pin(env, keys);
  jbyte* v = pin(env, vals);
  jlong* o = pin(env, voff);
  const int rc = kh_trie_open_host((const uint8_t*)k, (uint32_t)klen, (const uint8_t*)v, (const uint64_t*)o, n,
                                   (uint32_t)flags, root, &h);
  unpin_in(env, voff, o);
  unpin_in(env, vals, v);
  unpin_in(env, keys, k);
  if (rc != KH_OK) {
    throw_kh(env, rc);
    return 0;
  }
  if (rootOut) (*env)->SetByteArrayRegion(env, rootOut, 0, 32, (const jbyte*)root);
  return (jlong)(intptr_t)h;
}

/* MerklePatriciaTrie.apply(rootHash, source) (MerklePatriciaTrie.scala:60-66): open from a node
 * store (encodings enc[off[i]..off[i+1]), content addressed); a missing node throws
 * MPTNodeMissingException after writing its hash into missingOut (byte[32], nullable) */
JNIEXPORT jlong JNICALL Java_khipu_trie_gpu_Khst_openNodes(JNIEnv* env, jclass cls, jbyteArray root32,
                                                          jbyteArray enc, jlongArray off, jint flags,
                                                          jbyteArray missingOut) {
  (void)cls;
  const uint64_t n = count_of(env, off);
  uint8_t missing[32] = {0};
  kh_trie* h = NULL;
  jbyte* r = pin(env, root32);
  jbyte* e = pin(env, enc);
  jlong* o = pin(env, off);
  const int rc = kh_trie_open_nodes_host((const uint8_t*)r, (const uint8_t*)e, (const uint64_t*)o, n, (uint32_t)flags,
                                         missing, &h);
  unpin_in(env, off, o);
  unpin_in(env, enc, e);
  unpin_in(env, root32, r);
  if (rc == KH_ENODE && missingOut) (*env)->SetByteArrayRegion(env, missingOut, 0, 32, (const jbyte*)missing);
  if (rc != KH_OK) {
    throw_kh(env, rc);
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
  jbyte* k = pin(env, upKeys);
  jbyte* v = pin(env, upVals);
  jlong* o = pin(env, upVoff);
  jbyte* d = pin(env, delKeys);
  const int rc = kh_trie_apply_host(H(handle), (const uint8_t*)k, (const uint8_t*)v, (const uint64_t*)o, nup,
                                    (const uint8_t*)d, ndel, (uint32_t)klen, (uint32_t)flags, root, &st);
  unpin_in(env, delKeys, d);
  unpin_in(env, upVoff, o);
  unpin_in(env, upVals, v);
  unpin_in(env, upKeys, k);
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
  jint* ut = pin(env, upTrie);
  jbyte* k = pin(env, upKeys);
  jbyte* v = pin(env, upVals);
  jlong* o = pin(env, upVoff);
  jint* dt = pin(env, delTrie);
  jbyte* d = pin(env, delKeys);
  jint* to = pin(env, triesOut);
  jbyte* ro = pin(env, rootsOut);
  const int rc = kh_forest_apply_host(H(handle), (const uint32_t*)ut, (const uint8_t*)k, (const uint8_t*)v,
                                      (const uint64_t*)o, nup, (const uint32_t*)dt, (const uint8_t*)d, ndel,
                                      (uint32_t)klen, (uint32_t*)to, (uint8_t*)ro, cap, &nt, NULL);
  unpin_out(env, rootsOut, ro);
  unpin_out(env, triesOut, to);
  unpin_in(env, delKeys, d);
  unpin_in(env, delTrie, dt);
  unpin_in(env, upVoff, o);
  unpin_in(env, upVals, v);
  unpin_in(env, upKeys, k);
  unpin_in(env, upTrie, ut);
  if (rc == KH_ENOSPC) return -(jlong)nt;  /* committed; kh_forest_last_roots reads them again */
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
  jint* to = pin(env, triesOut);
  jbyte* ro = pin(env, rootsOut);
  const int rc = kh_forest_last_roots(H(handle), (uint32_t*)to, (uint8_t*)ro, cap, &nt);
  unpin_out(env, rootsOut, ro);
  unpin_out(env, triesOut, to);
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
  jint* st_ = pin(env, slotTrie);
  jbyte* sk = pin(env, slotKeys);
  jbyte* sv = pin(env, slotVals);
  jlong* so = pin(env, slotVoff);
  jint* sdt = pin(env, delSlotTrie);
  jbyte* sdk = pin(env, delSlotKeys);
  jbyte* ak = pin(env, accKeys);
  jbyte* av = pin(env, accBodies);
  jlong* ao = pin(env, accVoff);
  jint* at = pin(env, accTrie);
  jbyte* adk = pin(env, delAccKeys);
  const int rc = kh_block_commit_host(H(state), H(storage), (const uint32_t*)st_, (const uint8_t*)sk,
                                      (const uint8_t*)sv, (const uint64_t*)so, ns_up, (const uint32_t*)sdt,
                                      (const uint8_t*)sdk, ns_del, (uint32_t)slotKlen, (const uint8_t*)ak,
                                      (const uint8_t*)av, (const uint64_t*)ao, (const uint32_t*)at, na_up,
                                      (const uint8_t*)adk, na_del, (uint32_t)accKlen, root, &st);
  unpin_in(env, delAccKeys, adk);
  unpin_in(env, accTrie, at);
  unpin_in(env, accVoff, ao);
  unpin_in(env, accBodies, av);
  unpin_in(env, accKeys, ak);
  unpin_in(env, delSlotKeys, sdk);
  unpin_in(env, delSlotTrie, sdt);
  unpin_in(env, slotVoff, so);
  unpin_in(env, slotVals, sv);
  unpin_in(env, slotKeys, sk);
  unpin_in(env, slotTrie, st_);
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
  jbyte* hs = pin(env, hashes);
  jbyte* rl = pin(env, rlp);
  jlong* of = pin(env, off);
  const int rc = kh_trie_emit_nodes(H(handle), (uint8_t*)hs, cap, (uint8_t*)rl, rlp_cap, (uint64_t*)of, &nn, &nb);
  unpin_out(env, off, of);
  unpin_out(env, rlp, rl);
  unpin_out(env, hashes, hs);
  const jlong sz[2] = {(jlong)nn, (jlong)nb};
  if (sizes) (*env)->SetLongArrayRegion(env, sizes, 0, len_of(env, sizes) < 2 ? len_of(env, sizes) : 2, sz);
  if (rc == KH_ENOSPC) return -1;
  if (rc != KH_OK) {
    throw_kh(env, rc);
    return 0;
  }
  return (jlong)nn;
}

/* MerklePatriciaTrie.get for a batch (MerklePatriciaTrie.scala:90-147): byte[][] with null for
 * an absent key (None); trieIds (int[], nullable) for a forest */
JNIEXPORT jobjectArray JNICALL Java_khipu_trie_gpu_Khst_get(JNIEnv* env, jclass cls, jlong handle, jintArray trieIds,
                                                           jbyteArray keys, jint klen) {
  (void)cls;
  const jsize n = klen > 0 ? len_of(env, keys) / klen : 0;
  uint8_t* found = malloc((size_t)(n ? n : 1));
  uint64_t* voff = malloc(8 * ((size_t)n + 1));
  uint64_t need = 0, cap = 0;
  uint8_t* vals = NULL;
  int rc = KH_ENOSPC;
  if (!found || !voff) rc = KH_ENOMEM;
  for (int tries = 0; rc == KH_ENOSPC && tries < 2; ++tries) {  /* the first call reports the bytes needed */
    jbyte* k = pin(env, keys);
    jint* t = pin(env, trieIds);
    rc = kh_trie_get_host(H(handle), (const uint32_t*)t, (const uint8_t*)k, (uint32_t)klen, (uint64_t)n, vals, cap,
                          voff, found, &need);
    unpin_in(env, trieIds, t);
    unpin_in(env, keys, k);
    if (rc == KH_ENOSPC) {
      free(vals);
      vals = malloc((size_t)(need ? need : 1));
      cap = need;
      if (!vals) rc = KH_ENOMEM;
    }
  }
  jobjectArray out = NULL;
  if (rc == KH_OK) {
    out = (*env)->NewObjectArray(env, n, (*env)->FindClass(env, "[B"), NULL);
    for (jsize i = 0; out && i < n; ++i) {
      if (!found[i]) continue; /* None */
      jbyteArray v = bytes_of(env, vals + voff[i], (jsize)(voff[i + 1] - voff[i]));
      (*env)->SetObjectArrayElement(env, out, i, v);
      (*env)->DeleteLocalRef(env, v);
    }
  }
  free(vals);
  free(voff);
  free(found);
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
  jbyte* k = pin(env, upKeys);
  jbyte* v = pin(env, upVals);
  jlong* o = pin(env, upVoff);
  jbyte* d = pin(env, delKeys);
  const int rc = kh_trie_root_of_host(H(handle), (const uint8_t*)k, (const uint8_t*)v, (const uint64_t*)o, nup,
                                      (const uint8_t*)d, ndel, (uint32_t)klen, (uint32_t)flags, root, NULL);
  unpin_in(env, delKeys, d);
  unpin_in(env, upVoff, o);
  unpin_in(env, upVals, v);
  unpin_in(env, upKeys, k);
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
  const jsize n = len_of(env, usageOut);
  if (usageOut) (*env)->SetLongArrayRegion(env, usageOut, 0, n < 6 ? n : 6, v);
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
  const jsize n = len_of(env, beforeOut);
  if (beforeOut) (*env)->SetLongArrayRegion(env, beforeOut, 0, n < 2 ? n : 2, v);
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
  (*env)->SetLongArrayRegion(env, handleBox, 0, 1, &zero);  /* zeroed before the free: never freed twice */
  const int rc = kh_trie_free(H(h));
  if (rc != KH_OK) throw_kh(env, rc);
}
