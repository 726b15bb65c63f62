// ASan/UBSan driver (test infrastructure only): the CPU oracle
// (oracle/khipu_oracle.cc, oracle/batch_root.cc) and the host replay of the device
// per-thread code (tests/emu/khst_emu.cc: trie_ops.h, keccak.h, nodedata.h, synth.h)
// built with -fsanitize=address,undefined and run over random, adversarial and
// malformed inputs; roots are cross-checked so a silent miscompute also fails.
// Exit status 0 = clean; a sanitizer report aborts with a non-zero status.
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <map>
#include <random>
#include <string>
#include <vector>

extern "C" {
struct or_trie;
or_trie* or_trie_new();
void or_trie_free(or_trie*);
int or_trie_put(or_trie*, const uint8_t*, uint64_t, const uint8_t*, uint64_t);
int or_trie_remove(or_trie*, const uint8_t*, uint64_t);
void or_trie_root(or_trie*, uint8_t*);
void or_trie_persist(or_trie*);
void or_trie_reopen(or_trie*);
int or_node_children(const uint8_t*, uint64_t, int, uint8_t*, uint8_t*, uint32_t*);
int or_batch_roots(const uint8_t* keys, const uint64_t* koff, uint64_t klen, const uint8_t* vals, const uint64_t* voff,
                   uint64_t n, const uint64_t* seg_off, uint64_t nseg, int hash_keys, int nthreads, uint8_t* roots32,
                   uint64_t* stats);
int emu_build(const uint8_t* keys, const uint8_t* vals, const uint64_t* voff, uint64_t n, const uint32_t* seg,
              uint64_t nseg, uint32_t depth0, uint8_t* out_hash, uint32_t* out_len, uint8_t* out_inl,
              uint64_t* stats_out);
int emu_node_children(const uint8_t*, uint64_t, int, uint8_t*, uint8_t*, uint32_t*);
int emu_ansv_check(uint64_t seed, int iters);
void emu_synth(uint32_t cfg, uint64_t first, uint64_t n, uint8_t* addr, uint8_t* vals, uint64_t* voff);
}

static int fails = 0;
#define CHECK(c, ...)                         \
  do {                                        \
    if (!(c)) {                               \
      fprintf(stderr, "FAIL %s: ", #c);       \
      fprintf(stderr, __VA_ARGS__);           \
      fprintf(stderr, "\n");                  \
      ++fails;                                \
    }                                         \
  } while (0)

using Bytes = std::vector<uint8_t>;

struct Packed {
  Bytes k, v;
  std::vector<uint64_t> koff{0}, voff{0};
  void add(const Bytes& key, const Bytes& val) {
    k.insert(k.end(), key.begin(), key.end());
    v.insert(v.end(), val.begin(), val.end());
    koff.push_back(k.size());
    voff.push_back(v.size());
  }
  uint64_t n() const { return voff.size() - 1; }
};

static Bytes rand_bytes(std::mt19937_64& r, size_t n) {
  Bytes b(n);
  for (auto& x : b) x = (uint8_t)r();
  return b;
}

// sequential fold vs batch builder vs device-code replay (32-byte keys)
static void fixed_keys(uint64_t seed) {
  std::mt19937_64 r(seed);
  or_trie* t = or_trie_new();
  std::map<Bytes, Bytes> live;
  const int n = 300 + (int)(r() % 700);
  std::vector<Bytes> keys;
  for (int i = 0; i < n; ++i) {
    Bytes k = rand_bytes(r, 32);
    if (i && r() % 4 == 0) {  // share a long prefix with an earlier key (deep branches)
      const Bytes& o = keys[r() % keys.size()];
      size_t p = r() % 32;
      std::copy(o.begin(), o.begin() + p, k.begin());
    }
    keys.push_back(k);
    size_t vl = (r() % 5 == 0) ? 1 : 1 + r() % 200;
    Bytes v = rand_bytes(r, vl);
    if (or_trie_put(t, k.data(), 32, v.data(), v.size()) != 0) ++fails;
    live[k] = v;
    if (r() % 7 == 0) {  // a remove of a live or absent key
      const Bytes& d = r() % 2 ? keys[r() % keys.size()] : rand_bytes(r, 32);
      if (or_trie_remove(t, d.data(), 32) != 0) ++fails;
      live.erase(d);
    }
    if (r() % 50 == 0) {
      or_trie_persist(t);
      or_trie_reopen(t);
    }
  }
  uint8_t seq[32], bat[32], emu[32 * 1];
  or_trie_root(t, seq);
  or_trie_free(t);
  Packed P;
  for (auto& kv : live) P.add(kv.first, kv.second);
  uint64_t st[8];
  CHECK(or_batch_roots(P.k.data(), nullptr, 32, P.v.data(), P.voff.data(), P.n(), nullptr, 1, 0, 3, bat, st) == 0,
        "batch");
  CHECK(memcmp(seq, bat, 32) == 0, "seq vs batch seed %llu", (unsigned long long)seed);
  uint32_t len = 0;
  uint8_t inl[32];
  uint64_t est[8];
  CHECK(emu_build(P.k.data(), P.v.data(), P.voff.data(), P.n(), nullptr, 1, 0, emu, &len, inl, est) == 0, "emu");
  CHECK(memcmp(seq, emu, 32) == 0, "seq vs emu seed %llu", (unsigned long long)seed);
}

// variable-length keys (list tries, prefix keys): sequential fold vs batch builder
static void var_keys(uint64_t seed) {
  std::mt19937_64 r(seed);
  or_trie* t = or_trie_new();
  std::map<Bytes, Bytes> live;
  Bytes base = rand_bytes(r, 6);
  for (int i = 0; i < 400; ++i) {
    Bytes k(base.begin(), base.begin() + r() % 3);
    size_t L = r() % 6;
    for (size_t j = 0; j < L; ++j) k.push_back((uint8_t)(r() & 0x11));
    if (live.count(k)) continue;  // one put per key (the callers' contract)
    Bytes v = rand_bytes(r, 1 + r() % 60);
    or_trie_put(t, k.data(), k.size(), v.data(), v.size());
    live[k] = v;
  }
  uint8_t seq[32], bat[32];
  or_trie_root(t, seq);
  or_trie_free(t);
  Packed P;
  for (auto& kv : live) P.add(kv.first, kv.second);
  uint64_t st[8];
  CHECK(or_batch_roots(P.k.data(), P.koff.data(), 0, P.v.data(), P.voff.data(), P.n(), nullptr, 1, 0, 2, bat, st) == 0,
        "batch var");
  CHECK(memcmp(seq, bat, 32) == 0, "var seq vs batch seed %llu", (unsigned long long)seed);
}

// segmented synthetic accounts through the replay and the batch builder (hashed keys)
static void segmented_synth() {
  const uint64_t n = 6000;
  Bytes addr(20 * n), vals(n * 160);
  std::vector<uint64_t> voff(n + 1);
  emu_synth(3, 0, n, addr.data(), vals.data(), voff.data());
  std::vector<uint64_t> so = {0, 1, 2, 500, 500, 3000, n};
  uint64_t nseg = so.size() - 1;
  std::vector<uint8_t> roots(32 * nseg);
  uint64_t st[8];
  CHECK(or_batch_roots(addr.data(), nullptr, 20, vals.data(), voff.data(), n, so.data(), nseg, 1, 4, roots.data(),
                       st) == 0,
        "batch seg");
  // the same tries, one sequential fold each
  for (uint64_t s = 0; s < nseg; ++s) {
    Packed P;
    for (uint64_t i = so[s]; i < so[s + 1]; ++i)
      P.add(Bytes(addr.begin() + 20 * i, addr.begin() + 20 * i + 20),
            Bytes(vals.begin() + voff[i], vals.begin() + voff[i + 1]));
    uint8_t one[32];
    std::vector<uint64_t> so1 = {0, P.n()};
    CHECK(or_batch_roots(P.k.data(), nullptr, 20, P.v.data(), P.voff.data(), P.n(), so1.data(), 1, 1, 1, one, st) == 0,
          "batch one");
    CHECK(memcmp(one, roots.data() + 32 * s, 32) == 0, "segment %llu", (unsigned long long)s);
  }
}

// malformed / truncated / random node values through both decoders (memory safety only)
static void node_fuzz(uint64_t seed) {
  std::mt19937_64 r(seed);
  uint8_t o1[16 * 32 + 32], o2[16 * 32 + 32], k1[17], k2[17];
  uint32_t n1 = 0, n2 = 0;
  for (int it = 0; it < 20000; ++it) {
    size_t L = r() % 600;
    Bytes v = rand_bytes(r, L);
    if (L && r() % 2) v[0] = (uint8_t)(0xC0 + r() % 64);  // list headers more often
    if (L > 2 && r() % 3 == 0) v[1] = (uint8_t)(0x80 + r() % 64);
    int kind = (int)(r() % 3);
    or_node_children(v.data(), v.size(), kind, o1, k1, &n1);
    emu_node_children(v.data(), v.size(), kind, o2, k2, &n2);
  }
}

int main() {
  for (uint64_t s = 1; s <= 12; ++s) fixed_keys(s);
  for (uint64_t s = 1; s <= 8; ++s) var_keys(100 + s);
  segmented_synth();
  node_fuzz(7);
  CHECK(emu_ansv_check(3, 40) == 0, "ansv");
  if (fails) {
    fprintf(stderr, "%d checks failed\n", fails);
    return 1;
  }
  printf("sanitize: all checks clean\n");
  return 0;
}
