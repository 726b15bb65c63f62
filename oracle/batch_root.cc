// ORACLE — TEST INFRASTRUCTURE ONLY.
//
// Independent multi-threaded CPU batch state-root builder (SURVEY §7 step 2,
// §8(d) second baseline).  Used ONLY by tests/ and bench.py's cpu_baseline leg:
//   * as the full-size parity check of the GPU roots (the sequential oracle in
//     khipu_oracle.cc would need ~2 h for 100M accounts), and
//   * as the all-core CPU baseline.
// It shares no code with the device path (khipu_amd/csrc): its own Keccak, RLP,
// hex-prefix and topology, written from the reference semantics:
//   Keccak-256 legacy pad     crypto/hash/KeccakCore.scala:534-562, rate 136 (:570)
//   RLP                       rlp/RLP.scala:141-169
//   hex prefix                trie/HexPrefix.scala:11-21
//   node encodings            trie/Node.scala:21-44 (leaf, extension, branch + terminator)
//   inline-vs-hash            trie/Node.scala:110-115 (capped), :128-131, :158-163, :188-190
//   canonical shape           trie/MerklePatriciaTrie.scala:183-281 (put) and :430-477 (fix):
//                             a branch exactly where keys diverge, an extension exactly above
//                             a branch whose keys share more nibbles than the branch's depth,
//                             a key equal to a branch's prefix stored as that branch's value
//   root always hashed        MerklePatriciaTrie.scala:169; empty -> kec256(0x80) (trie/package.scala:41)
// Algorithm: sort the (key, input order) records, keep the last of equal keys (the
// foldLeft order of TrieAccounts.flush, TrieAccounts.scala:22-28), then a recursive
// divide over the sorted range: the common prefix of the range is the LCP of its first
// and last key.  Large tries are split into subtrees of at most T keys that run on a
// thread pool; the spine above them is assembled afterwards.  Keys may have any length
// (list tries: a key that is a prefix of another becomes a branch value).
#include <algorithm>
#include <atomic>
#include <cstdint>
#include <cstring>
#include <stdexcept>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

namespace brb {

// ---------------------------------------------------------------------------
// Keccak-f[1600] (FIPS 202 permutation), legacy 0x01 padding (KeccakCore.scala:537-546)
// ---------------------------------------------------------------------------
static const uint64_t RC[24] = {
    0x0000000000000001ULL, 0x0000000000008082ULL, 0x800000000000808AULL, 0x8000000080008000ULL,
    0x000000000000808BULL, 0x0000000080000001ULL, 0x8000000080008081ULL, 0x8000000000008009ULL,
    0x000000000000008AULL, 0x0000000000000088ULL, 0x0000000080008009ULL, 0x000000008000000AULL,
    0x000000008000808BULL, 0x800000000000008BULL, 0x8000000000008089ULL, 0x8000000000008003ULL,
    0x8000000000008002ULL, 0x8000000000000080ULL, 0x000000000000800AULL, 0x800000008000000AULL,
    0x8000000080008081ULL, 0x8000000000008080ULL, 0x0000000080000001ULL, 0x8000000080008008ULL};

static inline uint64_t rol(uint64_t x, int n) { return (x << n) | (x >> (64 - n)); }

// one round on named lanes (a[x + 5y]); the compiler keeps all 25 in registers
static inline void kf1600(uint64_t* s) {
  uint64_t a00 = s[0], a01 = s[1], a02 = s[2], a03 = s[3], a04 = s[4];
  uint64_t a05 = s[5], a06 = s[6], a07 = s[7], a08 = s[8], a09 = s[9];
  uint64_t a10 = s[10], a11 = s[11], a12 = s[12], a13 = s[13], a14 = s[14];
  uint64_t a15 = s[15], a16 = s[16], a17 = s[17], a18 = s[18], a19 = s[19];
  uint64_t a20 = s[20], a21 = s[21], a22 = s[22], a23 = s[23], a24 = s[24];
  for (int r = 0; r < 24; ++r) {
    uint64_t c0 = a00 ^ a05 ^ a10 ^ a15 ^ a20, c1 = a01 ^ a06 ^ a11 ^ a16 ^ a21;
    uint64_t c2 = a02 ^ a07 ^ a12 ^ a17 ^ a22, c3 = a03 ^ a08 ^ a13 ^ a18 ^ a23;
    uint64_t c4 = a04 ^ a09 ^ a14 ^ a19 ^ a24;
    uint64_t d0 = c4 ^ rol(c1, 1), d1 = c0 ^ rol(c2, 1), d2 = c1 ^ rol(c3, 1), d3 = c2 ^ rol(c4, 1),
             d4 = c3 ^ rol(c0, 1);
    // theta + rho + pi: b[y][2x+3y] = rot(a[x][y] ^ d[x], r[x][y])
    uint64_t b00 = a00 ^ d0;
    uint64_t b01 = rol(a06 ^ d1, 44), b02 = rol(a12 ^ d2, 43), b03 = rol(a18 ^ d3, 21), b04 = rol(a24 ^ d4, 14);
    uint64_t b05 = rol(a03 ^ d3, 28), b06 = rol(a09 ^ d4, 20), b07 = rol(a10 ^ d0, 3), b08 = rol(a16 ^ d1, 45),
             b09 = rol(a22 ^ d2, 61);
    uint64_t b10 = rol(a01 ^ d1, 1), b11 = rol(a07 ^ d2, 6), b12 = rol(a13 ^ d3, 25), b13 = rol(a19 ^ d4, 8),
             b14 = rol(a20 ^ d0, 18);
    uint64_t b15 = rol(a04 ^ d4, 27), b16 = rol(a05 ^ d0, 36), b17 = rol(a11 ^ d1, 10), b18 = rol(a17 ^ d2, 15),
             b19 = rol(a23 ^ d3, 56);
    uint64_t b20 = rol(a02 ^ d2, 62), b21 = rol(a08 ^ d3, 55), b22 = rol(a14 ^ d4, 39), b23 = rol(a15 ^ d0, 41),
             b24 = rol(a21 ^ d1, 2);
    // chi + iota
    a00 = b00 ^ (~b01 & b02) ^ RC[r]; a01 = b01 ^ (~b02 & b03); a02 = b02 ^ (~b03 & b04);
    a03 = b03 ^ (~b04 & b00); a04 = b04 ^ (~b00 & b01);
    a05 = b05 ^ (~b06 & b07); a06 = b06 ^ (~b07 & b08); a07 = b07 ^ (~b08 & b09);
    a08 = b08 ^ (~b09 & b05); a09 = b09 ^ (~b05 & b06);
    a10 = b10 ^ (~b11 & b12); a11 = b11 ^ (~b12 & b13); a12 = b12 ^ (~b13 & b14);
    a13 = b13 ^ (~b14 & b10); a14 = b14 ^ (~b10 & b11);
    a15 = b15 ^ (~b16 & b17); a16 = b16 ^ (~b17 & b18); a17 = b17 ^ (~b18 & b19);
    a18 = b18 ^ (~b19 & b15); a19 = b19 ^ (~b15 & b16);
    a20 = b20 ^ (~b21 & b22); a21 = b21 ^ (~b22 & b23); a22 = b22 ^ (~b23 & b24);
    a23 = b23 ^ (~b24 & b20); a24 = b24 ^ (~b20 & b21);
  }
  s[0] = a00; s[1] = a01; s[2] = a02; s[3] = a03; s[4] = a04;
  s[5] = a05; s[6] = a06; s[7] = a07; s[8] = a08; s[9] = a09;
  s[10] = a10; s[11] = a11; s[12] = a12; s[13] = a13; s[14] = a14;
  s[15] = a15; s[16] = a16; s[17] = a17; s[18] = a18; s[19] = a19;
  s[20] = a20; s[21] = a21; s[22] = a22; s[23] = a23; s[24] = a24;
}

// kec256 of len bytes; returns the permutations spent (floor(len/136)+1)
static uint32_t kec(const uint8_t* p, size_t len, uint8_t out[32]) {
  uint64_t s[25] = {0};
  uint32_t perms = 0;
  while (len >= 136) {
    for (int i = 0; i < 17; ++i) {
      uint64_t w;
      memcpy(&w, p + 8 * i, 8);
      s[i] ^= w;
    }
    kf1600(s);
    ++perms;
    p += 136;
    len -= 136;
  }
  uint8_t last[136] = {0};
  memcpy(last, p, len);
  last[len] ^= 0x01;
  last[135] ^= 0x80;
  for (int i = 0; i < 17; ++i) {
    uint64_t w;
    memcpy(&w, last + 8 * i, 8);
    s[i] ^= w;
  }
  kf1600(s);
  memcpy(out, s, 32);
  return perms + 1;
}

// ---------------------------------------------------------------------------
// RLP / hex-prefix writers into a flat byte buffer
// ---------------------------------------------------------------------------
struct Buf {
  uint8_t* p;
  size_t n = 0;
  void b(uint8_t x) { p[n++] = x; }
  void mem(const uint8_t* s, size_t k) {
    memcpy(p + n, s, k);
    n += k;
  }
};
static size_t be_len(size_t v) {
  size_t k = 0;
  for (; v; v >>= 8) ++k;
  return k;
}
static size_t hdr_len(size_t payload) { return payload < 56 ? 1 : 1 + be_len(payload); }
static void put_hdr(Buf& o, size_t payload, uint8_t base) {  // RLP.encodeLength (:157-169)
  if (payload < 56) {
    o.b((uint8_t)(base + payload));
    return;
  }
  size_t k = be_len(payload);
  o.b((uint8_t)(base + 55 + k));
  for (size_t i = k; i-- > 0;) o.b((uint8_t)(payload >> (8 * i)));
}
static size_t str_len(const uint8_t* s, size_t k) { return (k == 1 && s[0] < 0x80) ? 1 : hdr_len(k) + k; }
static void put_str(Buf& o, const uint8_t* s, size_t k) {  // RLP.scala:141-150
  if (k == 1 && s[0] < 0x80) {
    o.b(s[0]);
    return;
  }
  put_hdr(o, k, 0x80);
  o.mem(s, k);
}

// ---------------------------------------------------------------------------
// entries and nibbles
// ---------------------------------------------------------------------------
struct Ent {
  const uint8_t* k;
  uint32_t knib;  // key length in nibbles
  uint32_t vlen;
  const uint8_t* v;
};
static inline uint32_t nib(const Ent& e, uint32_t i) { return (e.k[i >> 1] >> ((i & 1) ? 0 : 4)) & 0xF; }
static uint32_t lcp_from(const Ent& a, const Ent& b, uint32_t d) {
  uint32_t m = a.knib < b.knib ? a.knib : b.knib;
  while (d < m && nib(a, d) == nib(b, d)) ++d;
  return d;
}

// hex prefix of nibbles [s, e) of key k (HexPrefix.scala:11-21) as an RLP string item
static size_t hp_bytes(uint32_t s, uint32_t e) { return (e - s) / 2 + 1; }
static void put_hp(Buf& o, const Ent& k, uint32_t s, uint32_t e, bool leaf) {
  uint32_t n = e - s;
  size_t h = n / 2 + 1;
  uint8_t first = (uint8_t)((2 * (leaf ? 1 : 0) + (n & 1)) << 4);
  uint32_t q = s;
  if (n & 1) first |= (uint8_t)nib(k, q++);
  if (h > 1) o.b((uint8_t)(0x80 + h));  // h < 56; a 1-byte HP (first < 0x80) is raw
  o.b(first);
  for (; q < e; q += 2) o.b((uint8_t)((nib(k, q) << 4) | nib(k, q + 1)));
}

// a capped reference: the encoding if < 32 B (embedded raw), else its hash
struct Ref {
  uint8_t len;  // 0 = empty child, 32 = hash, else inline encoding length
  uint8_t b[32];
};

struct Counters {
  uint64_t leaves = 0, branches = 0, exts = 0, hashes = 0, perms = 0, inl = 0;
  void add(const Counters& o) {
    leaves += o.leaves;
    branches += o.branches;
    exts += o.exts;
    hashes += o.hashes;
    perms += o.perms;
    inl += o.inl;
  }
};

struct Builder {
  const Ent* e;
  Counters c;
  const std::unordered_map<uint64_t, Ref>* memo = nullptr;  // precomputed subtrees by (hi << 32 | lo)
  std::vector<std::pair<size_t, std::pair<size_t, uint32_t>>>* tasks = nullptr;  // (lo, (hi, d)) collection
  size_t T = 0;

  // the node's encoding into enc (>= 600 B); returns its length
  Ref finish(const uint8_t* enc, size_t L, bool top) {
    Ref r;
    if (L < 32 && !top) {
      r.len = (uint8_t)L;
      memcpy(r.b, enc, L);
      ++c.inl;
      return r;
    }
    r.len = 32;
    c.perms += kec(enc, L, r.b);
    ++c.hashes;
    return r;
  }
  static size_t ref_enc_len(const Ref& r) { return r.len == 0 ? 1 : r.len == 32 ? 33 : r.len; }
  static void put_ref(Buf& o, const Ref& r) {
    if (r.len == 0)
      o.b(0x80);
    else if (r.len == 32) {
      o.b(0xA0);
      o.mem(r.b, 32);
    } else
      o.mem(r.b, r.len);  // an embedded node is its raw RLP list (Node.scala:28,34)
  }

  Ref leaf(size_t i, uint32_t d, bool top) {
    const Ent& x = e[i];
    ++c.leaves;
    uint8_t enc[64 + 4096];
    std::vector<uint8_t> big;
    uint8_t* p = enc;
    if (x.vlen > 4096) {
      big.resize(x.vlen + 128);
      p = big.data();
    }
    size_t h = hp_bytes(d, x.knib);
    size_t payload = (h == 1 ? 1 : 1 + h) + str_len(x.v, x.vlen);
    Buf o{p};
    put_hdr(o, payload, 0xC0);
    put_hp(o, x, d, x.knib, true);
    put_str(o, x.v, x.vlen);
    return finish(p, o.n, top);
  }

  Ref branch_at(size_t lo, size_t hi, uint32_t d, bool top) {
    ++c.branches;
    const Ent* val = nullptr;
    if (e[lo].knib == d) val = &e[lo++];  // the key equal to the prefix: the branch's value
    Ref ch[16];
    for (int q = 0; q < 16; ++q) ch[q].len = 0;
    size_t i = lo;
    while (i < hi) {
      uint32_t v = nib(e[i], d);
      size_t j = i + 1;
      while (j < hi && nib(e[j], d) == v) ++j;
      ch[v] = node(i, j, d + 1, false);
      i = j;
    }
    size_t payload = val ? str_len(val->v, val->vlen) : 1;
    for (int q = 0; q < 16; ++q) payload += ref_enc_len(ch[q]);
    std::vector<uint8_t> big;
    uint8_t enc[1024];
    uint8_t* p = enc;
    if (payload + 8 > sizeof enc) {
      big.resize(payload + 8);
      p = big.data();
    }
    Buf o{p};
    put_hdr(o, payload, 0xC0);
    for (int q = 0; q < 16; ++q) put_ref(o, ch[q]);
    if (val)
      put_str(o, val->v, val->vlen);
    else
      o.b(0x80);
    return finish(p, o.n, top);
  }

  Ref node(size_t lo, size_t hi, uint32_t d, bool top) {
    if (memo && !top && hi - lo <= T) {
      auto it = memo->find(((uint64_t)hi << 32) | lo);
      if (it != memo->end()) return it->second;
    }
    if (tasks && hi - lo <= T && !top) {
      tasks->push_back({lo, {hi, d}});
      return Ref{32, {0}};
    }
    if (hi - lo == 1) return leaf(lo, d, top);
    uint32_t p = lcp_from(e[lo], e[hi - 1], d);
    if (p == d) return branch_at(lo, hi, d, top);
    // extension [HP(nibbles d..p-1), ref(branch at p)] (Node.scala:24-28)
    ++c.exts;
    Ref br = branch_at(lo, hi, p, false);
    uint8_t enc[80];
    size_t h = hp_bytes(d, p);
    size_t payload = (h == 1 ? 1 : 1 + h) + ref_enc_len(br);
    Buf o{enc};
    put_hdr(o, payload, 0xC0);
    put_hp(o, e[lo], d, p, false);
    put_ref(o, br);
    return finish(enc, o.n, top);
  }
};

// sort + dedup one range of records [a, b) (indices into the input), entries out
static void sort_unique(std::vector<uint32_t>& idx, size_t a, size_t b, const std::vector<Ent>& in,
                        std::vector<Ent>& out, size_t* out_n) {
  auto less = [&](uint32_t x, uint32_t y) {
    const Ent& p = in[x];
    const Ent& q = in[y];
    uint32_t nb = (p.knib < q.knib ? p.knib : q.knib) / 2;
    int c = memcmp(p.k, q.k, nb);
    if (c) return c < 0;
    if (p.knib != q.knib) return p.knib < q.knib;
    return x < y;  // input order among equal keys
  };
  std::sort(idx.begin() + a, idx.begin() + b, less);
  size_t n = 0;
  for (size_t i = a; i < b; ++i) {
    const Ent& x = in[idx[i]];
    if (i + 1 < b) {
      const Ent& y = in[idx[i + 1]];
      if (x.knib == y.knib && memcmp(x.k, y.k, x.knib / 2) == 0) continue;  // a later put wins
    }
    out[a + n++] = x;
  }
  *out_n = n;
}

template <typename F>
static void parallel_for(size_t n, int nthreads, F f) {
  std::atomic<size_t> next{0};
  auto work = [&]() {
    for (size_t i; (i = next.fetch_add(1)) < n;) f(i);
  };
  std::vector<std::thread> th;
  int nt = nthreads < 1 ? 1 : nthreads;
  if ((size_t)nt > n) nt = (int)(n ? n : 1);
  for (int t = 1; t < nt; ++t) th.emplace_back(work);
  work();
  for (auto& t : th) t.join();
}

static const uint8_t EMPTY_TRIE[32] = {0x56, 0xe8, 0x1f, 0x17, 0x1b, 0xcc, 0x55, 0xa6, 0xff, 0x83, 0x45,
                                       0xe6, 0x92, 0xc0, 0xf8, 0x6e, 0x5b, 0x48, 0xe0, 0x1b, 0x99, 0x6c,
                                       0xad, 0xc0, 0x01, 0x62, 0x2f, 0xb5, 0xe3, 0x63, 0xb4, 0x21};

// Root of one trie over the unique sorted entries E[0, m), using nthreads for a large trie.
static void trie_root(const Ent* E, size_t m, int nthreads, uint8_t out[32], Counters& tot) {
  if (m == 0) {
    memcpy(out, EMPTY_TRIE, 32);
    return;
  }
  Builder b;
  b.e = E;
  size_t T = m / ((size_t)(nthreads > 0 ? nthreads : 1) * 64) + 1;
  if (nthreads <= 1 || m < 20000) {
    Ref r = b.node(0, m, 0, true);
    memcpy(out, r.b, 32);
    tot.add(b.c);
    return;
  }
  // 1) collect the subtrees of <= T keys hanging under the spine
  std::vector<std::pair<size_t, std::pair<size_t, uint32_t>>> tasks;
  {
    Builder s;
    s.e = E;
    s.tasks = &tasks;
    s.T = T < 2 ? 2 : T;
    s.node(0, m, 0, true);
  }
  // 2) compute them in parallel
  std::vector<Ref> res(tasks.size());
  std::vector<Counters> cs(tasks.size());
  parallel_for(tasks.size(), nthreads, [&](size_t t) {
    Builder w;
    w.e = E;
    res[t] = w.node(tasks[t].first, tasks[t].second.first, tasks[t].second.second, false);
    cs[t] = w.c;
  });
  std::unordered_map<uint64_t, Ref> memo;
  memo.reserve(tasks.size() * 2);
  for (size_t t = 0; t < tasks.size(); ++t) {
    memo[((uint64_t)tasks[t].second.first << 32) | tasks[t].first] = res[t];
    tot.add(cs[t]);
  }
  // 3) the spine, with the subtrees looked up
  b.memo = &memo;
  b.T = T < 2 ? 2 : T;
  Ref r = b.node(0, m, 0, true);
  memcpy(out, r.b, 32);
  tot.add(b.c);
}

}  // namespace brb

using namespace brb;

static thread_local std::string g_berr;

extern "C" {

const char* or_batch_last_error() { return g_berr.c_str(); }

// Roots of nseg independent tries (seg_off[nseg+1]; NULL = one trie over all n inputs).
//   keys: fixed klen bytes each (koff NULL) or packed keys[koff[i] .. koff[i+1])
//   hash_keys: trie key = kec256(key) (Address.hashedAddressEncoder / hashDataWordSerializable)
//   vals packed with voff[n+1] (absolute offsets into vals)
// stats (nullable, 8 x u64): leaves, branches, extensions, node hashes (>= 32 B + roots),
//   node perms, key perms, inline nodes, distinct keys.  Returns 0, or -1 with a message.
int or_batch_roots(const uint8_t* keys, const uint64_t* koff, uint64_t klen, const uint8_t* vals,
                   const uint64_t* voff, uint64_t n, const uint64_t* seg_off, uint64_t nseg, int hash_keys,
                   int nthreads, uint8_t* roots32, uint64_t* stats) {
  try {
    if (nthreads < 1) nthreads = 1;
    uint64_t one[2] = {0, n};
    if (!seg_off) {
      seg_off = one;
      nseg = 1;
    }
    // trie keys
    std::vector<uint8_t> hk;
    std::vector<Ent> in(n);
    std::atomic<uint64_t> kperms{0};
    if (hash_keys) {
      hk.resize(n * 32);
      parallel_for((n + 4095) / 4096, nthreads, [&](size_t blk) {
        uint64_t kp = 0;
        for (size_t i = blk * 4096; i < n && i < (blk + 1) * 4096; ++i) {
          const uint8_t* k = koff ? keys + koff[i] : keys + i * klen;
          size_t kl = koff ? koff[i + 1] - koff[i] : klen;
          kp += kec(k, kl, &hk[32 * i]);
        }
        kperms += kp;
      });
    }
    for (uint64_t i = 0; i < n; ++i) {
      Ent& x = in[i];
      if (hash_keys) {
        x.k = &hk[32 * i];
        x.knib = 64;
      } else {
        x.k = koff ? keys + koff[i] : keys + i * klen;
        size_t kl = koff ? koff[i + 1] - koff[i] : klen;
        if (kl > (1u << 20)) throw std::runtime_error("key length must be at most 2^20");
        x.knib = (uint32_t)(2 * kl);
      }
      x.v = vals + voff[i];
      x.vlen = (uint32_t)(voff[i + 1] - voff[i]);
    }
    std::vector<uint32_t> idx(n);
    for (uint64_t i = 0; i < n; ++i) idx[i] = (uint32_t)i;
    std::vector<Ent> srt(n);
    Counters tot;
    uint64_t distinct = 0;
    if (nseg == 1 && n > 100000 && nthreads > 1) {
      // bucket by the first key byte, sort the buckets in parallel, then one trie
      std::vector<uint64_t> cnt(257, 0);
      for (uint64_t i = 0; i < n; ++i) cnt[in[i].k[0] + 1]++;
      for (int q = 0; q < 256; ++q) cnt[q + 1] += cnt[q];
      std::vector<uint64_t> pos(cnt.begin(), cnt.end() - 1);
      for (uint64_t i = 0; i < n; ++i) idx[pos[in[i].k[0]]++] = (uint32_t)i;
      std::vector<size_t> un(256, 0);
      parallel_for(256, nthreads, [&](size_t q) { sort_unique(idx, cnt[q], cnt[q + 1], in, srt, &un[q]); });
      size_t m = 0;
      for (int q = 0; q < 256; ++q) {
        if (m != cnt[q]) std::memmove(&srt[m], &srt[cnt[q]], un[q] * sizeof(Ent));
        m += un[q];
      }
      distinct = m;
      trie_root(srt.data(), m, nthreads, roots32, tot);
    } else {
      std::vector<Counters> cs(nseg);
      std::vector<size_t> un(nseg, 0);
      if (seg_off[0] != 0 || seg_off[nseg] != n) throw std::runtime_error("seg_off must run from 0 to n");
      for (uint64_t s = 0; s < nseg; ++s)
        if (seg_off[s + 1] < seg_off[s]) throw std::runtime_error("seg_off not monotone");
      parallel_for(nseg, nthreads, [&](size_t s) {
        size_t a = seg_off[s], b = seg_off[s + 1];
        sort_unique(idx, a, b, in, srt, &un[s]);
        trie_root(srt.data() + a, un[s], nseg == 1 ? nthreads : 1, roots32 + 32 * s, cs[s]);
      });
      for (uint64_t s = 0; s < nseg; ++s) {
        tot.add(cs[s]);
        distinct += un[s];
      }
    }
    if (stats) {
      stats[0] = tot.leaves;
      stats[1] = tot.branches;
      stats[2] = tot.exts;
      stats[3] = tot.hashes;
      stats[4] = tot.perms;
      stats[5] = kperms.load();
      stats[6] = tot.inl;
      stats[7] = distinct;
    }
    return 0;
  } catch (std::exception& ex) {
    g_berr = ex.what();
    return -1;
  }
}

// kec256 through this file's own permutation (cross-checked against the oracle's in tests)
void or_batch_kec256(const uint8_t* in, uint64_t len, uint8_t* out32) { kec(in, (size_t)len, out32); }

}  // extern "C"
