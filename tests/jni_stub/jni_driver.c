/* TEST INFRASTRUCTURE ONLY: runs jni/khst_jni.c's wrappers through the in-process JNIEnv of
 * fake_env.c and prints one JSON object per check.
 *
 *   jni_driver cpu           argument checks that never reach the device (non-direct or short
 *                            buffers, a short root hash) and the empty trie
 *   jni_driver gpu FILE      FILE: u32 klen, u64 n, keys[n*klen], u64 voff[n+1], vals: the root
 *                            through trieRoot (arrays) and trieRootDirect (direct buffers);
 *                            openHost + get (present and absent keys) + free; openNodes over an
 *                            empty store (MPTNodeMissingException through Khst.nodeMissing) */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "fake_env.h"
#include "khst.h"

jbyteArray Java_khipu_trie_gpu_Khst_trieRoot(JNIEnv*, jclass, jbyteArray, jint, jbyteArray, jlongArray, jint, jlongArray);
jbyteArray Java_khipu_trie_gpu_Khst_trieRootDirect(JNIEnv*, jclass, jobject, jint, jobject, jobject, jlong, jint,
                                                   jlongArray);
jlong Java_khipu_trie_gpu_Khst_openNodes(JNIEnv*, jclass, jbyteArray, jbyteArray, jlongArray, jint, jbyteArray);
jlong Java_khipu_trie_gpu_Khst_openHost(JNIEnv*, jclass, jbyteArray, jint, jbyteArray, jlongArray, jint, jbyteArray);
jobjectArray Java_khipu_trie_gpu_Khst_get(JNIEnv*, jclass, jlong, jintArray, jbyteArray, jint);
void Java_khipu_trie_gpu_Khst_free(JNIEnv*, jclass, jlongArray);

static void hex(const uint8_t* p, int n, char* out) {
  for (int i = 0; i < n; ++i) sprintf(out + 2 * i, "%02x", p[i]);
  out[2 * n] = 0;
}
static void report(const char* check, jobject r) {
  char h[65] = "";
  FakeObj* o = (FakeObj*)r;
  if (o && o->kind == FK_ARRAY && o->len == 32) hex(o->data, 32, h);
  printf("{\"check\":\"%s\",\"root\":\"%s\",\"pending\":%d,\"exc\":\"%s\"}\n", check, h, fake.pending, fake.exc_class);
}

static int cpu_checks(void) {
  JNIEnv* env = fake_env();
  uint8_t keys[64] = {1}, vals[8] = {2};
  uint64_t voff[3] = {0, 4, 8};
  FakeObj* karr = fake_array(64, 1, keys);
  /* keys handed as a heap array to the direct wrapper */
  jobject r = Java_khipu_trie_gpu_Khst_trieRootDirect(env, NULL, (jobject)karr, 32, (jobject)fake_direct(vals, 8),
                                                      (jobject)fake_direct(voff, 24), 2, 0, NULL);
  report("direct_keys_not_direct", r);
  env = fake_env();
  r = Java_khipu_trie_gpu_Khst_trieRootDirect(env, NULL, (jobject)fake_direct(keys, 64), 32,
                                              (jobject)fake_direct(vals, 8), (jobject)fake_direct(voff, 16), 2, 0, NULL);
  report("direct_voff_short", r);
  env = fake_env();
  r = Java_khipu_trie_gpu_Khst_trieRootDirect(env, NULL, (jobject)fake_direct(keys, 64), 32,
                                              (jobject)fake_direct(vals, 7), (jobject)fake_direct(voff, 24), 2, 0, NULL);
  report("direct_vals_short", r);
  env = fake_env();
  r = Java_khipu_trie_gpu_Khst_trieRootDirect(env, NULL, NULL, 32, NULL, (jobject)fake_direct(voff, 8), 0, 0, NULL);
  report("direct_empty", r);
  env = fake_env();
  const uint64_t z = 0;
  r = Java_khipu_trie_gpu_Khst_trieRoot(env, NULL, (jbyteArray)fake_array(0, 1, NULL), 32,
                                        (jbyteArray)fake_array(0, 1, NULL), (jlongArray)fake_array(1, 8, &z), 0, NULL);
  report("array_empty", r);
  env = fake_env();
  jlong h = Java_khipu_trie_gpu_Khst_openNodes(env, NULL, (jbyteArray)fake_array(31, 1, keys),
                                               (jbyteArray)fake_array(0, 1, NULL), (jlongArray)fake_array(1, 8, &z), 0,
                                               NULL);
  printf("{\"check\":\"open_nodes_short_root\",\"handle\":%lld,\"pending\":%d,\"exc\":\"%s\"}\n", (long long)h,
         fake.pending, fake.exc_class);
  return 0;
}

static int gpu_checks(const char* path) {
  FILE* f = fopen(path, "rb");
  if (!f) return 2;
  uint32_t klen = 0;
  uint64_t n = 0;
  if (fread(&klen, 4, 1, f) != 1 || fread(&n, 8, 1, f) != 1) return 2;
  uint8_t* keys = malloc(n * klen + 1);
  uint64_t* voff = malloc(8 * (n + 1));
  if (fread(keys, klen, n, f) != n || fread(voff, 8, n + 1, f) != n + 1) return 2;
  uint8_t* vals = malloc(voff[n] + 1);
  if (fread(vals, 1, voff[n], f) != voff[n]) return 2;
  fclose(f);
  const uint32_t flags = klen == 32 ? 0 : KH_HASH_KEYS;
  FakeObj* ka = fake_array((jsize)(n * klen), 1, keys);
  FakeObj* va = fake_array((jsize)voff[n], 1, vals);
  FakeObj* oa = fake_array((jsize)(n + 1), 8, voff);
  JNIEnv* env = fake_env();
  jobject r = Java_khipu_trie_gpu_Khst_trieRoot(env, NULL, (jbyteArray)ka, (jint)klen, (jbyteArray)va, (jlongArray)oa,
                                                (jint)flags, NULL);
  report("array_root", r);
  env = fake_env();
  r = Java_khipu_trie_gpu_Khst_trieRootDirect(env, NULL, (jobject)fake_direct(keys, (jlong)(n * klen)), (jint)klen,
                                              (jobject)fake_direct(vals, (jlong)voff[n]),
                                              (jobject)fake_direct(voff, (jlong)(8 * (n + 1))), (jlong)n, (jint)flags,
                                              NULL);
  report("direct_root", r);
  /* open + get: the first 8 keys and one absent key */
  env = fake_env();
  FakeObj* rootOut = fake_array(32, 1, NULL);
  jlong h = Java_khipu_trie_gpu_Khst_openHost(env, NULL, (jbyteArray)ka, (jint)klen, (jbyteArray)va, (jlongArray)oa,
                                              (jint)flags, (jbyteArray)rootOut);
  char rh[65];
  hex(rootOut->data, 32, rh);
  printf("{\"check\":\"open_host\",\"root\":\"%s\",\"handle_ok\":%d,\"pending\":%d}\n", rh, h != 0, fake.pending);
  const uint32_t nq = n < 8 ? (uint32_t)n : 8;
  uint8_t* q = calloc(nq + 1, klen);
  memcpy(q, keys, (size_t)nq * klen);
  for (uint32_t b = 0; b < klen; ++b) q[(size_t)nq * klen + b] = (uint8_t)(0xA5 ^ b);
  env = fake_env();
  jobjectArray got = Java_khipu_trie_gpu_Khst_get(env, NULL, h, NULL, (jbyteArray)fake_array((jsize)((nq + 1) * klen), 1, q),
                                                  (jint)klen);
  int ok = got != NULL && !fake.pending;
  for (uint32_t i = 0; ok && i <= nq; ++i) {
    FakeObj* v = ((FakeObj**)((FakeObj*)got)->data)[i];
    if (i == nq) {
      ok = v == NULL;
      break;
    }
    /* the last put of a repeated key wins: find it */
    uint64_t last = n;
    for (uint64_t j = 0; j < n; ++j)
      if (!memcmp(keys + j * klen, q + (size_t)i * klen, klen)) last = j;
    ok = v && last < n && (uint64_t)v->len == voff[last + 1] - voff[last] &&
         !memcmp(v->data, vals + voff[last], (size_t)v->len);
  }
  printf("{\"check\":\"get\",\"ok\":%d,\"pending\":%d,\"exc\":\"%s\"}\n", ok, fake.pending, fake.exc_class);
  jlong box[1] = {h};
  FakeObj* ba = fake_array(1, 8, box);
  env = fake_env();
  Java_khipu_trie_gpu_Khst_free(env, NULL, (jlongArray)ba);
  Java_khipu_trie_gpu_Khst_free(env, NULL, (jlongArray)ba); /* idempotent */
  printf("{\"check\":\"free\",\"box\":%lld,\"pending\":%d}\n", (long long)((jlong*)ba->data)[0], fake.pending);
  /* a trie whose root is not in the (empty) node store */
  uint8_t missing[32];
  for (int i = 0; i < 32; ++i) missing[i] = (uint8_t)(0x11 * (i + 1));
  const uint64_t z = 0;
  env = fake_env();
  FakeObj* mo = fake_array(32, 1, NULL);
  jlong h2 = Java_khipu_trie_gpu_Khst_openNodes(env, NULL, (jbyteArray)fake_array(32, 1, missing),
                                                (jbyteArray)fake_array(0, 1, NULL), (jlongArray)fake_array(1, 8, &z), 0,
                                                (jbyteArray)mo);
  char mh[65], fh[65];
  hex(mo->data, 32, mh);
  hex(fake.node_missing_hash, 32, fh);
  printf("{\"check\":\"open_nodes_missing\",\"handle\":%lld,\"pending\":%d,\"exc\":\"%s\",\"factory_calls\":%d,"
         "\"factory_hash\":\"%s\",\"missing_out\":\"%s\"}\n",
         (long long)h2, fake.pending, fake.exc_class, fake.node_missing_calls, fh, mh);
  return 0;
}

int main(int argc, char** argv) {
  if (argc >= 2 && !strcmp(argv[1], "cpu")) return cpu_checks();
  if (argc >= 3 && !strcmp(argv[1], "gpu")) return gpu_checks(argv[2]);
  fprintf(stderr, "usage: jni_driver cpu | gpu FILE\n");
  return 2;
}
