// Resident forest: the nodes of one or many tries kept in HBM between commits
// (SURVEY §8 rows f1 incremental commit, f2 per-block write-back, a12 many storage
// tries per block, a10 open from a node store).
//
// The reference keeps a trie as immutable node objects found by hash through
// NodeStorage (MerklePatriciaTrie.scala:520-542) and re-hashes the root path of every
// put / remove (:157-477), one key at a time, from TrieAccounts.flush /
// TrieStorage.flush (TrieAccounts.scala:22-28, TrieStorage.scala:43-60).  Here every
// node of the current version is a RECORD found by its ANCHOR: (trie id, the depth d
// in nibbles at which the node hangs, the key's first d nibbles).  A leaf's record holds
// its key and the value's place in a value heap; a branch's record (with the extension
// above it, if any: anchor d < branch depth db) holds a key under it, db, its child
// nibble mask and two capped references (the branch's, and the one its parent sees).
// The anchor -> record map is an open-addressing table (64-bit tags, linear probing,
// tombstones; the record is checked on every tag match).
//
// A commit (a block's dirty set, all tries at once):
//   1. descend: every op walks down from its trie's root by anchor lookups; every
//      branch it passes into is OPENED, the leaf it ends at is TOUCHED
//      (MerklePatriciaTrie.put/remove's search path);
//   2. gather ELEMENTS: the untouched children of opened branches (unchanged subtrees:
//      a leaf, or a branch kept as one opaque element with its cached reference), the
//      touched leaves no op replaced or deleted, and every upsert;
//   3. an element build (run_build): sort, topology, and hashing of exactly the nodes
//      on the dirty paths -- the canonical shape put / fix converge to (:183-477) -- with
//      subtree elements referenced, or re-wrapped in a new extension when their anchor
//      moved;
//   4. the new nodes replace the opened ones in the map; the nodes whose encodings
//      changed are the block's write-back set.
// Work per commit is O(dirty keys x depth x 16), not O(resident keys).
#pragma once
#include "keyorder.h"
#include "nodedata.h"

namespace khst {

KH_HD uint64_t fmix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
  return z ^ (z >> 31);
}

// word q of a key restricted to its first d nibbles (the rest zero)
KH_HD uint64_t prefix_word(const uint64_t* key, uint32_t d, int q) {
  const uint32_t nib0 = 16u * (uint32_t)q;
  if (d <= nib0) return 0;
  uint64_t w = key[q];
  if (d >= nib0 + 16) return w;
  uint64_t be = bswap64(w);
  be &= ~0ULL << (64 - 4 * (d - nib0));
  return bswap64(be);
}
KH_HD bool prefix_eq(const uint64_t* a, const uint64_t* b, uint32_t d) {
  for (int q = 0; q < 4; ++q)
    if (prefix_word(a, d, q) != prefix_word(b, d, q)) return false;
  return true;
}
KH_HD uint64_t anchor_tag(uint32_t t, uint32_t d, const uint64_t* key) {
  uint64_t h = fmix64(((uint64_t)t << 8) ^ d ^ 0x9E3779B97F4A7C15ULL);
  for (int q = 0; q < 4; ++q) h = fmix64(h ^ prefix_word(key, d, q) ^ (0x632BE59BD9B4E019ULL * (q + 1)));
  return h | 2;  // 0 = empty slot, 1 = tombstone
}
// the key with nibble i set to v
KH_HD void set_nibble(uint64_t* key, uint32_t i, uint32_t v) {
  const int q = (int)(i >> 4);
  const uint32_t byte = (i >> 1) & 7, sh = 8 * byte + ((i & 1) ? 0 : 4);
  key[q] = (key[q] & ~(0xFULL << sh)) | ((uint64_t)v << sh);
}

// ---- khipu's value-only branch.  A re-put of a 32-byte key whose leaf hangs under a
// depth-63 branch (its remaining path empty) goes through putInLeafNode with ml == 0 and an
// empty existing key: BranchNode.withValueOnly, then putInBranchNode with an empty key sets
// the value (MerklePatriciaTrie.scala:187-199, 258-262).  The leaf becomes a branch at depth 64
// with no children and the new value -- not the canonical trie of the same keys, but khipu's.
// Here it is a record with db = VB_DEPTH (no branch of 32-byte keys sits at depth 64), mask 0
// and its value span; in an element build it is a subtree element whose capped reference is
// that of its encoding [0x80 x 16, value].  Removing its key throws in khipu (fix of a branch
// with no children and no value, :430-477): the commit is refused.
constexpr uint32_t VB_DEPTH = 64;
KH_HD uint32_t vb_put_len(uint8_t* out, uint32_t p, uint64_t len, uint32_t base) {  // RLP length prefix
  if (len < 56) {
    out[p++] = (uint8_t)(base + len);
    return p;
  }
  const uint32_t nb = be_nbytes(len);
  out[p++] = (uint8_t)(base + 55 + nb);
  for (uint32_t i = nb; i-- > 0;) out[p++] = (uint8_t)(len >> (8 * i));
  return p;
}
// the encoding of a value-only branch holding val (<= vl + 26 bytes); returns its length
KH_HD uint32_t vb_encode(const uint8_t* val, uint32_t vl, uint8_t* out) {
  const uint32_t v0 = vl ? val[0] : 0;
  uint32_t p = vb_put_len(out, 0, 16 + rlp_str_len(vl, v0), 0xC0);
  for (int c = 0; c < 16; ++c) out[p++] = 0x80;
  if (!(vl == 1 && v0 < 0x80)) p = vb_put_len(out, p, vl, 0x80);
  for (uint32_t i = 0; i < vl; ++i) out[p++] = val[i];
  return p;
}

constexpr uint8_t REC_DEAD = 0, REC_LIVE = 1;

// Node records: one 128-byte record per node (array of structures), so a probe's check
// (trie, anchor depth, key) and a descent step read ONE 64-byte line, and a whole record
// (an element of the next build) two; round 3's twelve arrays cost up to twelve lines per
// record (the block-commit gather: profiles/r3x_block_commit_timeline_50m.json).
//   [0, 32)  k: a key under the node (a leaf: its key)
//   32 t (u32) trie id | 36 d: anchor depth | 37 db: EL_LEAF or the branch depth |
//   38 mask (u16): branch child nibbles | 40 live | 41 rl | 42 brl | 44 vl (u32) |
//   48 vo (u64): leaf value offset in the heap
//   [64, 96)  ref: capped reference the parent holds (the extension's, if any); rl its length
//   [96, 128) bref: a branch's own capped reference; brl its length
// The accessors keep the structure-of-arrays indexing of the code that uses them: R.rt[r],
// and word q of the key R.rk[4 * r + q] (R.key(r) is the key's address).
constexpr uint64_t REC_BYTES = 128;
template <typename T, uint32_t OFF>
struct RecField {
  uint8_t* b;
  KH_HD T& operator[](uint64_t r) const { return *(T*)(b + r * REC_BYTES + OFF); }
};
template <uint32_t OFF>
struct RecWords {  // 4 words per record: index 4 r + q
  uint8_t* b;
  KH_HD uint64_t& operator[](uint64_t i) const { return *(uint64_t*)(b + (i >> 2) * REC_BYTES + OFF + (i & 3) * 8); }
};
struct Recs {
  RecWords<0> rk;
  RecField<uint32_t, 32> rt;
  RecField<uint8_t, 36> rd;
  RecField<uint8_t, 37> rdb;
  RecField<uint16_t, 38> rmask;
  RecField<uint8_t, 40> rlive;
  RecField<uint8_t, 41> rrl;
  RecField<uint8_t, 42> rbrl;
  RecField<uint32_t, 44> rvl;
  RecField<uint64_t, 48> rvo;
  RecWords<64> rref;
  RecWords<96> rbref;
  KH_HD uint64_t* key(uint64_t r) const { return (uint64_t*)(rk.b + r * REC_BYTES); }
};
// one whole record, composed in registers and written as 16-byte stores (a record written
// field by field across a wave touches one line per field and lane)
struct RecVal {
  uint64_t k[4];
  uint32_t t;
  uint8_t d, db;
  uint16_t mask;
  uint8_t live, rl, brl;
  uint32_t vl;
  uint64_t vo;
  uint64_t ref[4], bref[4];
};
KH_HD void rec_store(uint8_t* base, uint64_t r, const RecVal& v) {
  uint64_t w[16];
  for (int q = 0; q < 4; ++q) {
    w[q] = v.k[q];
    w[8 + q] = v.ref[q];
    w[12 + q] = v.bref[q];
  }
  w[4] = (uint64_t)v.t | ((uint64_t)v.d << 32) | ((uint64_t)v.db << 40) | ((uint64_t)v.mask << 48);
  w[5] = (uint64_t)v.live | ((uint64_t)v.rl << 8) | ((uint64_t)v.brl << 16) | ((uint64_t)v.vl << 32);
  w[6] = v.vo;
  w[7] = 0;
#ifdef __HIP_DEVICE_COMPILE__
  ulonglong2* d = (ulonglong2*)(base + r * REC_BYTES);
#pragma unroll
  for (int q = 0; q < 8; ++q) d[q] = make_ulonglong2(w[2 * q], w[2 * q + 1]);
#else
  memcpy(base + r * REC_BYTES, w, REC_BYTES);
#endif
}
KH_HD Recs recs_at(uint8_t* base) {
  return Recs{{base}, {base}, {base}, {base}, {base}, {base}, {base}, {base}, {base}, {base}, {base}, {base}};
}

// The anchor -> record map: 16-byte slots (tag, record) so a probe reads one line.
struct MapTag {
  uint8_t* b;
  KH_HD unsigned long long& operator[](uint64_t s) const { return *(unsigned long long*)(b + s * 16); }
};
struct MapRec {
  uint8_t* b;
  KH_HD uint32_t& operator[](uint64_t s) const { return *(uint32_t*)(b + s * 16 + 8); }
};
struct AMap {
  MapTag tag;    // [cap] 0 empty, 1 tombstone
  MapRec rec;
  uint64_t mask; // cap - 1 (cap a power of two, load <= 1/2 incl. tombstones)
};

KH_HD uint32_t map_find(const AMap& M, const Recs& R, uint32_t t, uint32_t d, const uint64_t* key) {
  const uint64_t h = anchor_tag(t, d, key);
  for (uint64_t s = h & M.mask, n = 0; n <= M.mask; s = (s + 1) & M.mask, ++n) {
    const uint64_t g = M.tag[s];
    if (g == 0) return NONE;
    if (g == h) {
      const uint32_t r = M.rec[s];
      if (R.rt[r] == t && R.rd[r] == d && prefix_eq(R.key(r), key, d)) return r;
    }
  }
  return NONE;
}
// slot of record r at its current anchor (NONE if absent)
KH_HD uint64_t map_slot_of(const AMap& M, const Recs& R, uint32_t r) {
  const uint64_t h = anchor_tag(R.rt[r], R.rd[r], R.key(r));
  for (uint64_t s = h & M.mask, n = 0; n <= M.mask; s = (s + 1) & M.mask, ++n) {
    const uint64_t g = M.tag[s];
    if (g == 0) return ~0ULL;
    if (g == h && M.rec[s] == r) return s;
  }
  return ~0ULL;
}

// MerklePatriciaTrie.get (MerklePatriciaTrie.scala:90-147) on the records: the anchor
// descent of a commit (a branch whose extension the key leaves, or an empty child
// anchor, ends the search); the leaf record holding exactly `key`, or NONE
KH_HD uint32_t forest_get(const AMap& M, const Recs& R, uint32_t t, const uint64_t* key) {
  uint32_t d = 0;
  for (int step = 0; step < 70; ++step) {
    const uint32_t r = map_find(M, R, t, d, key);
    if (r == NONE) return NONE;
    const uint32_t db = R.rdb[r];
    if (db == EL_LEAF || db == VB_DEPTH) {  // a leaf, or a value-only branch: it holds one key
      const uint64_t* L = R.key(r);
      return (L[0] == key[0] && L[1] == key[1] && L[2] == key[2] && L[3] == key[3]) ? r : NONE;
    }
    if (lcp_nibbles(load_key(key, 0), load_key(R.key(r), 0)) < (int)db) return NONE;  // leaves the extension
    d = db + 1;
  }
  return NONE;
}

// ---- the batch of ops, sorted by (trie, key), one op per key (the last one wins)
enum : uint8_t { FOP_UPSERT = 1, FOP_DELETE = 2 };
struct FOps {
  const uint64_t* key;  // [n*4]
  const uint32_t* trie; // [n]
  const uint8_t* kind;  // [n]
  uint64_t n;
};

// elements of an element build
struct Elems {
  uint64_t* key;    // [cap*4]
  uint32_t* seg;    // compact trie index of the build (segment id)
  uint8_t* db;      // EL_LEAF or branch depth
  uint64_t* bref;   // [cap*4]
  uint8_t* brl;
  uint64_t* vo;     // value offset in the heap (leaves)
  uint32_t* vl;
  uint32_t* src;    // source record, NONE for an upsert
  uint8_t* oldd;    // the source record's anchor depth (EL_NEW for an upsert)
  uint64_t* cref;   // [cap*4] the source record's capped reference (rref)
  uint8_t* crl;
  uint8_t* late;    // its value arrives late (FCommit::late; upserts only)
  unsigned long long* n;  // counter
  uint64_t cap;
};

KH_HD uint32_t seg_of(const uint32_t* tries, uint32_t nt, uint32_t t) {
  uint32_t lo = 0, hi = nt;
  while (lo < hi) {
    uint32_t mid = (lo + hi) >> 1;
    if (tries[mid] < t) lo = mid + 1; else hi = mid;
  }
  return lo;
}

KH_HD void elem_fill(const Recs& R, uint32_t r, uint32_t seg, const Elems& E, uint64_t e);
template <typename PushFn>
KH_HD void elem_from_record(const Recs& R, uint32_t r, uint32_t seg, const Elems& E, PushFn push) {
  elem_fill(R, r, seg, E, push());
}
// element e from record r (e claimed from E.n by the caller)
KH_HD void elem_fill(const Recs& R, uint32_t r, uint32_t seg, const Elems& E, uint64_t e) {
  if (e >= E.cap) return;  // the host sized the buffer; overflow flagged by the counter
  for (int q = 0; q < 4; ++q) E.key[4 * e + q] = R.rk[4ull * r + q];
  E.seg[e] = seg;
  E.db[e] = R.rdb[r];
  for (int q = 0; q < 4; ++q) E.bref[4 * e + q] = R.rbref[4ull * r + q];
  E.brl[e] = R.rbrl[r];
  E.vo[e] = R.rvo[r];
  E.vl[e] = (R.rdb[r] == EL_LEAF || R.rdb[r] == VB_DEPTH) ? R.rvl[r] : 0;  // (a value-only branch keeps its value)
  E.src[e] = r;
  E.oldd[e] = R.rd[r];
  for (int q = 0; q < 4; ++q) E.cref[4 * e + q] = R.rref[4ull * r + q];
  E.crl[e] = R.rrl[r];
  E.late[e] = 0;
}


// ---- open a resident trie from (root hash, node store):
// MerklePatriciaTrie.apply(rootHash, source) + getNode (MerklePatriciaTrie.scala:60-66,
// 520-542; Node.nodeDec, Node.scala:46-102): the nodes reachable from the root are
// decoded level by level on the device into records.  A frontier item is one node to
// decode: referenced by hash (looked up in the store) or embedded (its < 32-byte
// encoding carried in the item).
struct OItems {
  uint64_t* pre;   // [cap*4] key prefix: nibbles [0, d) of every key below
  uint8_t* a;      // anchor depth of the record the node belongs to
  uint8_t* d;      // depth at which the node starts (> a: the child of an extension)
  uint64_t* ref;   // [cap*4] hash, or the embedded encoding
  uint8_t* rl;     // 32 = hash, else the embedded length
  uint64_t* pref;  // [cap*4] the capped reference the record's parent holds
  uint8_t* prl;
  unsigned long long* n;
  uint64_t cap;
};
struct NStore {
  const uint64_t* hash;  // [m*4] sorted node hashes
  const uint32_t* idx;   // [m] node index of sorted hash i
  uint64_t m;
  const uint8_t* enc;
  const uint64_t* off;   // [n+1]
};
enum : unsigned long long { OPEN_OK = 0, OPEN_MISSING = 1, OPEN_BAD = 2, OPEN_VALUE = 3 };

KH_HD void hp_nibbles(const uint8_t* b, uint32_t len, uint32_t* n, bool* leaf, uint8_t* out) {
  // HexPrefix.decode (HexPrefix.scala:30-40): flag nibble, optional pad nibble
  const uint32_t f = b[0] >> 4;
  *leaf = (f & 2) != 0;
  // *n is the FULL nibble count (it may exceed 64: the caller rejects such a path); only the
  // first 64 nibbles are written to out
  uint32_t k = 0;
  if (f & 1) out[k++] = b[0] & 0xF;
  for (uint32_t i = 1; i < len; ++i) {
    if (k < 64) out[k] = b[i] >> 4;
    if (k + 1 < 64) out[k + 1] = b[i] & 0xF;
    k += 2;
  }
  *n = k;
}
KH_HD void words_of(const uint8_t* p, uint32_t len, uint64_t w[4]) {  // <= 32 bytes, zero padded
  for (int q = 0; q < 4; ++q) w[q] = 0;
  for (uint32_t i = 0; i < len && i < 32; ++i) w[i >> 3] |= (uint64_t)p[i] << (8 * (i & 7));
}

}  // namespace khst
