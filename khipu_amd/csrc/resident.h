// Incremental commit over a resident trie.
//
// The reference folds a block's dirty set into the trie one key at a time:
// TrieAccounts.flush / TrieStorage.flush (TrieAccounts.scala:22-28,
// TrieStorage.scala:43-60) call MerklePatriciaTrie.put / remove
// (MerklePatriciaTrie.scala:157-281, 290-477), and every call re-encodes and
// re-hashes the whole root path.  The trie after the fold is the canonical trie of
// the final (key, value) set, so the batch path here:
//   1. sorts the batch (upserts, then deletes; the last op on a key wins),
//   2. merges it into the resident sorted (key, value) arrays (ops below),
//   3. rebuilds the topology of the merged set (O(n) memory passes, no sort),
//   4. re-hashes only the DIRTY branches: those whose key prefix (d nibbles) is a
//      prefix of some changed key (updated, inserted or deleted) — exactly the
//      nodes the reference's put/remove paths touch.  A clean branch covers the same
//      key set as before, so its reference is looked up in the previous version's
//      tables (by its first key and depth) instead of being recomputed.  A leaf is
//      re-encoded only if it was inserted or upserted or its path changed (parent
//      depth); otherwise its previous reference is carried over.
// Per-element ops (KH_HD): the HIP kernels and the host replay share them.
#pragma once
#include "trie_ops.h"

namespace khst {

// lexicographic compare of two 32-byte keys held as 4 little-endian words
KH_HD int key_cmp(const uint64_t* a, const uint64_t* b) {
  for (int j = 0; j < 4; ++j) {
    uint64_t x = bswap64(a[j]), y = bswap64(b[j]);
    if (x != y) return x < y ? -1 : 1;
  }
  return 0;
}

// first index in sorted keys[0, n) not less than k
KH_HD uint64_t key_lower_bound(const uint64_t* keys, uint64_t n, const uint64_t* k) {
  uint64_t lo = 0, hi = n;
  while (lo < hi) {
    uint64_t mid = (lo + hi) >> 1;
    if (key_cmp(keys + 4 * mid, k) < 0)
      lo = mid + 1;
    else
      hi = mid;
  }
  return lo;
}

enum OpKind : uint8_t { OP_NOP = 0, OP_UPD = 1, OP_INS = 2, OP_DEL = 3 };

struct Merge {
  // resident version
  const uint64_t* rkey;  // [m*4] sorted, unique
  const uint64_t* roff;  // [m+1] value offsets into rval
  uint64_t m;
  // the batch, sorted by key and deduplicated (the last op on a key kept)
  const uint64_t* okey;  // [nops*4]
  const uint32_t* oidx;  // [nops] input op index: < nup upsert, else delete
  uint64_t nops, nup;
  const uint64_t* uoff;  // [nup+1] upsert value offsets
  // per op
  uint32_t* o_lb;    // lower bound in rkey
  uint8_t* o_kind;   // OpKind
  uint32_t* o_ins;   // 1 if insert (scanned in place to the insert rank)
  uint32_t* o_eff;   // 1 if the op changes the trie (scanned to the dirty-key slot)
  // per resident position (m+1 entries)
  uint32_t* pos_ins;  // inserts with this lower bound (scanned: inserts before)
  uint32_t* pos_del;  // 1 if deleted (scanned: deletes before)
  uint32_t* pos_cnt;  // raw insert counts (kept for the inclusive term)
  uint32_t* pos_upd;  // sorted-op slot updating this position, or NONE
  // merged version
  uint64_t* nkey;    // [m'*4]
  uint32_t* nlen;    // [m'] value length
  uint64_t* nsrc;    // [m'] value source offset; bit 63: the upsert buffer
  uint32_t* oldpos;  // [m'] resident position of the key, NONE if inserted
  uint8_t* nupd;     // [m'] 1 if the value comes from the batch (updated or inserted)
  uint64_t* dkey;    // [ndirty*4] changed keys, sorted
};

constexpr uint64_t SRC_UPSERT = 1ULL << 63;

// 1. classify op o against the resident keys
KH_HD void op_locate(const Merge& M, uint64_t o) {
  const uint64_t* k = M.okey + 4 * o;
  uint64_t lb = key_lower_bound(M.rkey, M.m, k);
  bool found = lb < M.m && key_cmp(M.rkey + 4 * lb, k) == 0;
  bool up = M.oidx[o] < M.nup;
  uint8_t kind = up ? (found ? OP_UPD : OP_INS) : (found ? OP_DEL : OP_NOP);
  M.o_lb[o] = (uint32_t)lb;
  M.o_kind[o] = kind;
  M.o_ins[o] = kind == OP_INS ? 1u : 0u;
  M.o_eff[o] = kind != OP_NOP ? 1u : 0u;
}

// 2. mark resident positions (device: pos_cnt via atomicAdd — several inserts can
// share a lower bound; the host replay passes a plain increment)
template <typename AddFn>
KH_HD void op_mark(const Merge& M, uint64_t o, AddFn add) {
  uint32_t lb = M.o_lb[o];
  switch (M.o_kind[o]) {
    case OP_INS: add(&M.pos_cnt[lb]); break;
    case OP_DEL: M.pos_del[lb] = 1; break;
    case OP_UPD: M.pos_upd[lb] = (uint32_t)o; break;
    default: break;
  }
}

// 3a. place resident key j (after the scans: pos_ins = exclusive scan of pos_cnt,
// pos_del = exclusive scan of the delete flags, del_flag = the raw flags)
KH_HD void op_place_resident(const Merge& M, const uint32_t* del_flag, uint64_t j) {
  if (del_flag[j]) return;
  uint64_t np = j - M.pos_del[j] + M.pos_ins[j] + M.pos_cnt[j];
  for (int q = 0; q < 4; ++q) M.nkey[4 * np + q] = M.rkey[4 * j + q];
  uint32_t u = M.pos_upd[j];
  if (u != NONE) {
    uint32_t src = M.oidx[u];
    M.nsrc[np] = SRC_UPSERT | M.uoff[src];
    M.nlen[np] = (uint32_t)(M.uoff[src + 1] - M.uoff[src]);
  } else {
    M.nsrc[np] = M.roff[j];
    M.nlen[np] = (uint32_t)(M.roff[j + 1] - M.roff[j]);
  }
  M.oldpos[np] = (uint32_t)j;
  M.nupd[np] = u != NONE ? 1 : 0;
}

// 3b. place inserted op o (o_ins scanned to the insert rank) and record the dirty
// key of every effective op (o_eff scanned to its slot)
KH_HD void op_place_op(const Merge& M, const uint32_t* ins_flag, const uint32_t* eff_flag, uint64_t o) {
  if (eff_flag[o]) {
    uint64_t s = M.o_eff[o];
    for (int q = 0; q < 4; ++q) M.dkey[4 * s + q] = M.okey[4 * o + q];
  }
  if (!ins_flag[o]) return;
  uint32_t lb = M.o_lb[o];
  uint64_t np = (uint64_t)lb - M.pos_del[lb] + M.o_ins[o];
  for (int q = 0; q < 4; ++q) M.nkey[4 * np + q] = M.okey[4 * o + q];
  uint32_t src = M.oidx[o];
  M.nsrc[np] = SRC_UPSERT | M.uoff[src];
  M.nlen[np] = (uint32_t)(M.uoff[src + 1] - M.uoff[src]);
  M.oldpos[np] = NONE;
  M.nupd[np] = 1;
}

// ---- dirty marking and clean-branch lookup (after the topology of the merged set)

// The previous version's tables, enough to find a clean branch's reference.
struct Prev {
  Pyr P;                  // its boundary LCP pyramid (level 0 = u)
  const uint32_t* bid;    // [nb] scanned rep flags: branch id at a group's first boundary
  const uint64_t* ref;    // [B*4] capped reference of each branch node (extension excluded)
  const uint32_t* rlen;   // [B] its encoding length
  uint64_t nb;            // boundaries (m - 1)
  const uint32_t* oldpos; // merged position -> previous position
  const uint8_t* upd;     // merged position -> value upserted
  const int8_t* lpd;      // previous leaves' parent depths
  const uint64_t* lref;   // previous leaves' capped references
  const uint32_t* lrlen;
};

// branch j is dirty iff some changed key starts with its d-nibble prefix
KH_HD void op_br_dirty(const Topo& T, const uint64_t* dkey, uint64_t nd, uint32_t j) {
  uint64_t f = T.br_first[j];
  uint32_t d = T.br_depth[j];
  Key4 k = load_key(T.skey, f);
  // smallest key with this prefix: nibbles >= d cleared
  uint64_t lo[4] = {k.w0, k.w1, k.w2, k.w3};
  for (int q = 0; q < 4; ++q) {
    uint32_t nib0 = 16u * q;  // nibbles [nib0, nib0+16) live in word q (big-endian order)
    if (d <= nib0) {
      lo[q] = 0;
    } else if (d < nib0 + 16) {
      uint32_t keep = d - nib0;  // leading nibbles kept
      uint64_t be = bswap64(lo[q]);
      be &= ~0ULL << (64 - 4 * keep);
      lo[q] = bswap64(be);
    }
  }
  uint64_t i = key_lower_bound(dkey, nd, lo);
  bool dirty = false;
  if (i < nd) {
    Key4 x = load_key(dkey, i);
    dirty = lcp_nibbles(x, k) >= (int)d;
  }
  T.br_dirty[j] = dirty ? 1 : 0;
}

// a clean branch: same keys as a branch of the previous version at the same depth
// starting at the same key -> copy that branch's reference.  Its group's first
// boundary is the first boundary >= its first leaf with LCP+1 < d+2.
KH_HD void op_br_clean(const Topo& T, const Prev& V, uint32_t j) {
  if (T.br_dirty[j]) return;
  uint32_t f = V.oldpos[T.br_first[j]];
  uint32_t t = (uint32_t)T.br_depth[j] + 2;
  int64_t b = -1;
  if (f != NONE && f < V.nb) b = V.P.lv[0][f] < t ? (int64_t)f : ansv_right(V.P, f, t);
  if (b < 0 || V.P.lv[0][b] != t - 1) {  // cannot happen for a clean branch
    T.ctr[CTR_ERR] = 2;
    return;
  }
  uint32_t ob = V.bid[b];
  for (int q = 0; q < 4; ++q) T.br_ref[4 * j + q] = V.ref[4 * ob + q];
  T.br_rlen[j] = V.rlen[ob];
}

}  // namespace khst
