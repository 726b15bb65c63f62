// Per-element operations of the batch state-root pipeline.  Each function is the
// body of one GPU thread (kernels in khst.hip call them with their global thread
// index); they are __host__ __device__ so tests/emu can replay the exact same
// code on the CPU against the oracle.
//
// Trie shape from sorted keys (no pointer chasing).  Sorted distinct keys
// K_0 < ... < K_{m-1}; boundary b (between K_b and K_{b+1}) carries
//   u[b] = LCP_nibbles(K_b, K_{b+1}) + 1, or 0 at a segment break.
// A branch node is a maximal run of boundaries with equal u and only larger u
// between them (its "group"); its depth is u-1, its children are the key
// ranges the group's boundaries separate, so a branch with k children has k-1
// boundaries.  The group's leftmost boundary (rep) is the one whose previous
// smaller-or-equal boundary (PSE) is strictly smaller.  A node spanning keys
// [s, e] hangs under the group of the larger of u[s-1], u[e] (its parent), at
// child ordinal ord[s-1]+1 or ord[e].  An extension sits between a branch at
// depth d and its parent at depth pd when d > pd+1 (nibbles pd+1 .. d-1); a
// leaf's path is nibbles pd+1 .. 63.  This reproduces exactly the canonical
// trie that khipu's sequential put/fix builds (MerklePatriciaTrie.scala:157-281,
// 430-477): branches only where keys diverge, extensions only above branches.
//
// Node encodings (trie/Node.scala:21-44, rlp/RLP.scala:116-169,
// trie/HexPrefix.scala:11-21): leaf = [HP(path, leaf), value],
// extension = [HP(shared, ext), ref], branch = [ref_0 .. ref_15, ""]; a child
// is referenced by its kec256 when its encoding is >= 32 B, else embedded
// verbatim (Node.scala:114, 128-131, 158-163, 188-190).
#pragma once
#include "keccak.h"

namespace khst {

constexpr uint32_t NONE = 0xFFFFFFFFu;

// ---- key helpers (keys: 4 little-endian u64 words = the 32 key bytes in order)
struct Key4 {
  uint64_t w0, w1, w2, w3;
};
KH_HD Key4 load_key(const uint64_t* k, uint64_t i) {
  const uint64_t* p = k + 4 * i;
  return Key4{p[0], p[1], p[2], p[3]};
}
KH_HD uint64_t key_word(const Key4& k, int j) { return j == 0 ? k.w0 : j == 1 ? k.w1 : j == 2 ? k.w2 : k.w3; }
KH_HD uint32_t key_byte(const Key4& k, int j) { return (uint32_t)(key_word(k, j >> 3) >> (8 * (j & 7))) & 0xFF; }
KH_HD uint32_t key_nibble(const Key4& k, int i) {
  uint32_t b = key_byte(k, i >> 1);
  return (i & 1) ? (b & 0xF) : (b >> 4);
}
KH_HD uint64_t bswap64(uint64_t x) {
#ifdef __HIPCC__
  return __builtin_bswap64(x);
#else
  return __builtin_bswap64(x);
#endif
}
KH_HD int clz64(uint64_t x) { return x ? __builtin_clzll(x) : 64; }

// Number of equal leading nibbles of two keys (64 if equal).
KH_HD int lcp_nibbles(const Key4& a, const Key4& b) {
  uint64_t x;
  if ((x = a.w0 ^ b.w0)) return clz64(bswap64(x)) >> 2;
  if ((x = a.w1 ^ b.w1)) return 16 + (clz64(bswap64(x)) >> 2);
  if ((x = a.w2 ^ b.w2)) return 32 + (clz64(bswap64(x)) >> 2);
  if ((x = a.w3 ^ b.w3)) return 48 + (clz64(bswap64(x)) >> 2);
  return 64;
}

// ---- RLP length helpers (RLP.scala:157-169)
KH_HD uint32_t be_nbytes(uint64_t v) {
  uint32_t n = 0;
  while (v) {
    ++n;
    v >>= 8;
  }
  return n;
}
KH_HD uint32_t rlp_hdr_len(uint64_t payload) { return payload < 56 ? 1 : 1 + be_nbytes(payload); }
// encoded length of an RLP string of len bytes whose first byte is b0
KH_HD uint64_t rlp_str_len(uint64_t len, uint32_t b0) {
  if (len == 1 && b0 < 0x80) return 1;
  return rlp_hdr_len(len) + len;
}

// ---- byte writer into an 8-byte-aligned buffer (whole-word stores); consecutive
// words are `stride` words apart (1: packed; m: the transposed leaf layout)
struct BW {
  uint64_t* dst;
  uint64_t acc;
  uint32_t fill;
  uint64_t stride;
  KH_HD BW(uint64_t* d, uint64_t s = 1) : dst(d), acc(0), fill(0), stride(s) {}
  KH_HD void put(uint64_t w, uint32_t nb) {  // nb in [1, 8]; low nb bytes of w
    w &= low_bytes_mask(nb);
    acc |= w << (8 * fill);
    uint32_t nf = fill + nb;
    if (nf >= 8) {
      *dst = acc;
      dst += stride;
      acc = fill ? (w >> (8 * (8 - fill))) : 0;
      nf -= 8;
    }
    fill = nf;
  }
  KH_HD void put1(uint32_t b) { put(b, 1); }
  KH_HD void flush() {
    if (fill) *dst = acc;
  }
  KH_HD void flush_or() {  // the rest of the last word already holds bytes written elsewhere
    if (fill) *dst = (*dst & ~low_bytes_mask(fill)) | acc;
  }
  KH_HD void len_prefix(uint64_t len, uint32_t offset) {  // RLP.encodeLength
    if (len < 56) {
      put1((uint32_t)(len + offset));
    } else {
      uint32_t nb = be_nbytes(len);
      put1(nb + offset + 55);
      for (int i = (int)nb - 1; i >= 0; --i) put1((uint32_t)(len >> (8 * i)) & 0xFF);
    }
  }
  // copy key bytes [from, to)
  KH_HD void key_suffix(const Key4& k, uint32_t from, uint32_t to = 32) {
    while (from < to) {
      uint32_t nb = 8 - (from & 7);
      if (nb > to - from) nb = to - from;
      put(key_word(k, from >> 3) >> (8 * (from & 7)), nb);
      from += nb;
    }
  }
  // copy n bytes from an arbitrary global address
  KH_HD void bytes(const uint8_t* p, uint64_t n) {
    while (n) {
      uint32_t nb = n < 8 ? (uint32_t)n : 8;
      put(load64u_n(p, nb), nb);
      p += nb;
      n -= nb;
    }
  }
  // copy n (< 32) bytes held little-endian in 4 words
  KH_HD void words(const uint64_t* w, uint32_t n) {
    for (int j = 0; j < 4 && n; ++j) {
      uint32_t nb = n < 8 ? n : 8;
      put(w[j], nb);
      n -= nb;
    }
  }
};

// ---------------------------------------------------------------------------
// Build state shared by all stages (device pointers; sizes in comments).
// ---------------------------------------------------------------------------
struct Topo {
  uint64_t m;        // distinct keys (leaves)
  uint32_t depth0;   // 0: whole tries; 1: top-nibble subtries (shard unit)
  uint32_t segmented;
  const uint64_t* skey;   // [m*4] sorted keys
  const uint32_t* sidx;   // [m] input index of sorted key i
  const uint32_t* sseg;   // [m] segment id (segmented only)
  const uint8_t* kn;      // [m] key length in nibbles (variable-length key builds; nullable: 64)
  const uint32_t* sck;    // [m] sorted 32-bit sort words (plain builds; nullable): the segment id in the
                          //     top ck_sb bits, then the big-endian leading key bits; the sorted keys are
                          //     never gathered (sorted_key reads the input keys past these bits)
  uint32_t ck_sb;         // segment bits at the top of sck (0: unsegmented)
  const uint8_t* vals;    // input values
  const uint64_t* voff;   // [n+1] (or [n] offsets with vlen_in)
  const uint32_t* vlen_in; // [n] value lengths (nullable: voff[i+1] - voff[i])
  uint64_t* svoff;        // [m] value offset of sorted key i (gathered once after the sort)
  uint32_t* svlen;        // [m] value length of sorted key i
  uint8_t* u;             // [m-1] boundary values
  int32_t* psv;           // [m-1] previous strictly smaller boundary (-1: none)
  int32_t* nsv;           // [m-1] next strictly smaller boundary (-1: none)
  int32_t* pse;           // [m-1] previous boundary of the same group (its smaller-or-equal neighbour
                          //       when that carries the same value; -1: the group's first)
  uint32_t* rep;          // [m-1] group representative of b
  uint8_t* ord;           // [m-1] ordinal of b within its group
  uint32_t* isrep_bid;     // [m-1] 1 if rep, then (after scan) branch id of rep
  // early builds with tiles (nullable): the representative flags as bits (bit b % 32 of
  // word b / 32), written per wave by the tile kernel; a representative's branch id is
  // rep_pref[b / 32] + the set bits below it (bid_of).  isrep_bid is not used then: the 100M-entry
  // flag array and its scan (a write, a read, a read + write) beside the leaf kernel become 12.5 MB
  uint32_t* rep_bits;
  const uint32_t* rep_pref;  // [words + 1] exclusive prefix of the words' popcounts
  const uint32_t* bid_pos;  // nullable: isrep_bid holds key-order ids, their level positions (leaf-position builds skip k_bid_remap)
  uint8_t* glast;         // [nb] 1 unless a later boundary of the same group exists (preset 1)
  uint8_t* gk;            // [nb] at a group's representative: its branch's child count
  // branches (B <= m-1)
  uint32_t* br_k;         // child count
  uint32_t* br_cbase;     // first child record
  uint8_t* br_depth;
  uint8_t* br_ext;        // extension nibbles above the branch (0: none)
  uint32_t* br_parent;    // parent branch id or NONE (top of a segment)
  uint8_t* br_pord;       // ordinal in parent
  uint32_t* br_first;     // first key index of the branch's range
  uint64_t* br_aoff;      // position of the branch in the level order (message slot)
  uint32_t* br_len;       // encoding length of the branch
  uint32_t* ex_len;       // encoding length of the extension
  // leaves
  uint32_t* lf_parent;
  uint8_t* lf_pord;
  int8_t* lf_pd;          // parent depth (depth0-1 for a top leaf)
  uint64_t* lf_aoff;      // long leaves (> 135 B): aligned length, scanned into the
                          // offset in the packed long-leaf region at `arena`
  uint64_t* lmsg;         // one-block leaves: word q of leaf i at lmsg[q * lstride + i]
  uint64_t lstride;       //   (transposed: a wave's store / load of word q is contiguous)
  uint32_t* lf_len;
  // child references: 32 B each + meta (len | nibble << 8); len 32 = hash
  uint64_t* cref;
  uint16_t* cmeta;
  // per-node hashes for write-back emission (nullable)
  uint64_t* lf_hash;
  uint64_t* br_hash;
  uint64_t* ex_hash;
  // message stores
  uint8_t* arena;          // long leaves (> 135 B), packed
  uint64_t* bmsg;          // branch messages: level d's t-th branch, word q at
                           //   bmsg[BR_WORDS * lb[d] + q * cnt_d + t]  (transposed per level)
  uint64_t* xmsg;          // extension messages, same scheme with EXT_WORDS
  const uint32_t* lb;      // [65] first order position of each depth (lb[64] = B)
  // capped references kept for a resident forest's records (element builds; nullable)
  uint64_t* br_ref;    // [B*4] capped reference of each branch node
  uint32_t* br_rlen;   // [B] its encoding length
  uint64_t* lf_ref;    // [m*4] capped reference of each element node (leaf or extension)
  uint32_t* lf_rlen;   // [m]
  // early leaves (plain root builds; nullable): capped reference and its length
  // (32 = hash, EMETA_LONG = not hashed yet: longer than one Keccak block)
  uint64_t* lf_eref;   // [m*4]
  uint8_t* lf_emeta;   // [m] preset to 32 (a hash): only inline and long leaves write theirs
  const uint64_t* kin; // [n*4] the keys in input order (the early leaf kernel reads them sequentially)
  uint64_t* pdinv;     // [n] per INPUT position: parent depth << 32 | sorted position; PDINV_SKIP for
                       //     a dropped duplicate
  uint64_t* lf_dst;    // [m] nibble << 56 | parent child-record slot, LINK_TOP for a top leaf (op_leaf_link;
                       //     segmented builds)
  // leaf positions (default for unsegmented plain root builds): the leaves write no child
  // records.  A branch child's record carries CM_BR and the end of its key range (cend), so
  // the parent walks its range and finds each leaf child at the next sorted position, whose
  // stash (lf_eref / lf_emeta) is the reference (op_branch_stream, op_leaf_children)
  uint32_t lpos;       // set before the leaf kernel: a top leaf publishes its result itself
  uint32_t lf_inline;  // some leaf is inline (else every leaf child is a 32-byte hash)
  uint32_t* br_end;    // [B] one past the last sorted key of the branch's range (nullable)
  uint32_t* cend;      // [C] at a branch child's record: that branch's br_end (nullable: no positions)
  uint32_t lvl_nsh;    // per level launch: 28 - 4 * the level's depth (a leaf child's nibble in sck)
  uint32_t lvl_depth;  //   and the depth itself (deeper levels: the nibble from the input key)
  uint32_t* longlist;  // [m] sorted leaves longer than one Keccak block (the leaf kernel lists them)
  uint32_t* wlist;     // [B] per level launch: the level's branches spanning >= T12_SPAN keys (k_branch_fused
  uint32_t* wcnt;      //   lists them for k_branch_wide), and their count (one per level launch, zeroed)
  // element builds (resident commits, forest.h; all nullable): an element is a leaf, or
  // a SUBTREE standing for an unchanged branch at depth el_db[i] whose capped reference
  // is el_bref / el_brl (its keys all share key i's first el_db nibbles)
  const uint8_t* el_db;     // [m] EL_LEAF or the subtree's branch depth
  const uint8_t* el_late;   // [n] nullable, INPUT order (via sidx): the element's value arrives late (two leaf passes)
  const uint64_t* el_bref;  // [m*4]
  const uint8_t* el_brl;    // [m]
  const uint8_t* el_oldd;   // [m] anchor depth of the element's node in the previous version (EL_NEW: none)
  const uint64_t* el_cref;  // [m*4] that node's capped reference (the parent's view)
  const uint8_t* el_crl;    // [m]
  uint64_t* ex_ref;         // [B*4] capped reference of each extension (nullable)
  uint32_t* ex_rlen;        // [B]
  const uint8_t* emit_sel;  // [m + 2B] node q is emitted iff set (nullable: every node >= 32 B + tops)
  // per-result outputs
  uint64_t* res_hash;  // [nres*4]
  uint32_t* res_len;   // [nres]
  uint64_t* res_inl;   // [nres*4]
  // counters
  unsigned long long* ctr;  // [0] node hashes, [1] node perms, [2] inline nodes, [3] arena bytes, [4] error
  uint32_t* depth_hist;     // [64]
};

enum {
  CTR_HASHES = 0, CTR_PERMS = 1, CTR_INLINE = 2, CTR_ARENA = 3, CTR_ERR = 4, CTR_EXT = 5, CTR_LONGB = 6,
  // (row 0; the stat shards use indices 0-2 and 5 of their rows)
  // scratch slots for device-side totals read back by the host
  CTR_NDUP = 7,  // sorts: repeated keys (k_tie_fix)
  CTR_TIE = 8, CTR_M = 9, CTR_B = 10, CTR_BRBYTES = 11, CTR_LFBYTES = 12, CTR_C = 13, CTR_E0 = 14, CTR_E1 = 15,
  CTR_N = 16
};
// The statistics counters (node hashes, permutations, inline nodes, extensions) are added
// by one atomic per block; with ~400k blocks per 100M-key kernel a single address
// serialises them, so they are spread over CTR_SHARDS rows of CTR_N (one 128-byte line
// each) by block index and summed on the host.  Row 0 holds every other counter.
constexpr int CTR_SHARDS = 64;
constexpr unsigned long long ERR_LEAF_TOPO = 9;  // CTR_ERR: a leaf's parent depth / sorted position out of range
constexpr int CTR_LONGN = 16 + 7;  // longlist length (row 1, index 7: unused by the stat shards)
constexpr int CTR_PYR = 16 + 8;    // k_pyramid's finished-block count (row 1, index 8)
constexpr int CTR_LIST = 16 + 9;   // element builds: the re-encoded leaves listed by k_leaf_prep
constexpr int CTR_TLIST = 16 + 10; // k_topo_tile's two list lengths (row 1, indices 10 and 11)
constexpr int CTR_LIST2 = 16 + 12; // element builds with late values: the late leaves' list (row 1, index 12)
// counter add returning the old value (the host replay is single-threaded)
KH_HD unsigned long long ctr_add(unsigned long long* p, unsigned long long v) {
#ifdef __HIP_DEVICE_COMPILE__
  return atomicAdd(p, v);
#else
  const unsigned long long o = *p;
  *p += v;
  return o;
#endif
}
KH_HD unsigned long long* ctr_stat(unsigned long long* ctr, int idx, uint32_t block) {
  return ctr + (uint64_t)(block % CTR_SHARDS) * CTR_N + idx;
}

constexpr uint32_t LEAF_SHORT_MAX = 135;  // one Keccak block: the transposed leaf layout
constexpr uint32_t LEAF_WORDS = 17;

KH_HD uint32_t branch_bound(uint32_t k) { return 24 + 32 * k; }  // >= 3 + 33k + (16-k) + 1, 8-aligned
constexpr uint32_t EXT_BOUND = 72;                               // >= 2 + 33 + 33
constexpr uint32_t BR_WORDS = 67;                                // branch_bound(16) / 8
constexpr uint32_t EXT_WORDS = EXT_BOUND / 8;

// message slot of branch j (its position g in the level order): word-0 pointer + stride
struct Slot {
  uint64_t* w;
  uint64_t stride;
};
KH_HD Slot branch_slot(const Topo& T, uint64_t g, uint32_t d, bool ext) {
  uint64_t first = T.lb[d], cnt = T.lb[d + 1] - first;
  uint64_t* base = ext ? T.xmsg + (uint64_t)EXT_WORDS * first : T.bmsg + (uint64_t)BR_WORDS * first;
  return Slot{base + (g - first), cnt};
}

// sorted key i where nibbles [0, need) are read: the gathered sorted keys, or on the
// unsegmented plain path (sck set, no sorted keys materialised) the first 8 nibbles from
// the sorted prefixes and, past them, the input key through its index
KH_HD Key4 sorted_key(const Topo& T, uint64_t i, uint32_t need) {
  if (!T.sck) return load_key(T.skey, i);
  if (need <= (32 - T.ck_sb) / 4) return Key4{bswap64((uint64_t)(T.sck[i] << T.ck_sb) << 32), 0, 0, 0};
  return load_key(T.kin, T.sidx[i]);
}

KH_HD uint32_t result_index(const Topo& T, uint64_t first_key) {
  if (T.segmented) return T.sseg[first_key];
  if (T.depth0 == 1) return (uint32_t)(sorted_key(T, first_key, 1).w0 & 0xFF) >> 4;
  return 0;
}

// ---- variable-length keys (list tries): key i has kn[i] nibbles; a key
// that is a prefix of the next ones is the VALUE of the branch at its own depth (the
// 17th slot, Node.scala:31-40), published to the parent as a value marker
constexpr uint16_t VAL_META = 0xFFFF;
KH_HD uint32_t key_nibs(const Topo& T, uint64_t i) { return T.kn ? T.kn[i] : 64; }
KH_HD bool is_branch_value(const Topo& T, uint64_t i) {
  return T.kn && T.lf_parent[i] != NONE && (int32_t)T.kn[i] == T.lf_pd[i];
}

// ---- element builds: subtree elements
constexpr uint8_t EL_LEAF = 0xFF, EL_NEW = 0xFF;
KH_HD bool el_subtree(const Topo& T, uint64_t i) { return T.el_db && T.el_db[i] != EL_LEAF; }
// an unchanged node still hanging at its old anchor: its encoding is what it was, so its
// cached reference is published as is (no re-encoding, no hash, nothing written back)
KH_HD bool el_cached(const Topo& T, uint64_t i, uint32_t a) { return T.el_oldd && T.el_oldd[i] == a; }
// encoding length of a subtree element hanging at anchor depth a: 0 extension nibbles ->
// no node of its own (the parent embeds / references the branch: returns its capped
// length); else the extension [HP(nibbles a .. db-1, ext), ref(branch)]
KH_HD uint32_t el_ext_nibbles(const Topo& T, uint64_t i, uint32_t a) {
  if (a > T.el_db[i]) {  // cannot happen (a subtree's neighbours diverge above its branch): flag it
    T.ctr[CTR_ERR] = 7;
    return 0;
  }
  return (uint32_t)T.el_db[i] - a;
}
KH_HD uint32_t ext_enc_len(uint32_t e, uint32_t brl) {
  uint32_t hl = e / 2 + 1;
  uint32_t xpay = (hl == 1 ? 1 : 1 + hl) + (brl >= 32 ? 33 : brl);
  return rlp_hdr_len(xpay) + xpay;
}

// ---- stage: boundary values
KH_HD uint8_t lcp_value(const Topo& T, uint64_t b) {
  int l;
  if (T.sck) {  // the first 8 nibbles from the sorted prefixes; the input keys only past them
    const uint32_t x = (T.sck[b] ^ T.sck[b + 1]) << T.ck_sb;  // the key bits (a segment break: v = 0 below)
    l = x ? (int)((uint32_t)clz64((uint64_t)x << 32) >> 2)
          : lcp_nibbles(load_key(T.kin, T.sidx[b]), load_key(T.kin, T.sidx[b + 1]));
  } else {
    l = lcp_nibbles(load_key(T.skey, b), load_key(T.skey, b + 1));
  }
  if (T.kn) {  // padded keys: the common prefix ends with the shorter key
    if (l > (int)T.kn[b]) l = T.kn[b];
    if (l > (int)T.kn[b + 1]) l = T.kn[b + 1];
  }
  uint8_t v = (uint8_t)(l + 1);
  if (l < (int)T.depth0 || l > 63) v = 0;  // 64 cannot occur after dedup
  if (T.segmented && T.sseg[b] != T.sseg[b + 1]) v = 0;
  return v;
}
KH_HD void op_lcp(const Topo& T, uint64_t b) { T.u[b] = lcp_value(T, b); }
// the early leaves' scatter record of sorted leaf i from its two boundary values
// A boundary value outside 0 / depth0 + 1 .. 64 (stale bytes: round 5's r5y fault, where a
// speculative build's unvalued tie run left the bytes of an earlier build, leaf depths fell
// outside 0..63 and the leaf kernel indexed past its buffers) is flagged (CTR_ERR =
// ERR_LEAF_TOPO: the build returns KH_EINTERNAL at the topology's counter sync, before any
// branch level) and clamped, so the leaf kernel never reads a depth out of range.  Guarded here,
// where the depths are made (every early-leaf record passes through this function), not in the
// leaf kernel: the same check there cost 10 % of its time (a changed register allocation).
KH_HD void pd_scatter_vals(const Topo& T, uint64_t i, uint32_t va, uint32_t vc) {
  uint32_t v = va > vc ? va : vc;
  if (v > 64 || (v != 0 && v < T.depth0 + 1)) {
    T.ctr[CTR_ERR] = ERR_LEAF_TOPO;
    v = 0;
  }
  const int32_t pd = v == 0 ? (int32_t)T.depth0 - 1 : (int32_t)v - 1;
  T.pdinv[T.sidx ? T.sidx[i] : i] = ((uint64_t)(uint8_t)(int8_t)pd << 32) | i;
}

// ---- stage: all nearest smaller values over a 64-ary min pyramid
struct Pyr {
  const uint8_t* lv[8];
  uint64_t sz[8];
  int nl;
};

// SWAR helpers: 8 boundary values (each <= 64 < 128) per 64-bit word.
// lt_mask(x, t): bit 7 of byte i set iff byte i of x < t, exactly, for bytes <= 127
// and t in [1, 128]: (x_i | 0x80) - t never borrows across bytes.
KH_HD uint64_t lt_mask(uint64_t x, uint32_t t) {
  const uint64_t ones = 0x0101010101010101ULL, highs = 0x8080808080808080ULL;
  return ~((x | highs) - ones * t) & highs;
}
KH_HD int ctz64(uint64_t x) { return x ? __builtin_ctzll(x) : 64; }
// bytes [lo, hi) of an 8-byte group as a byte-lane mask of bit 7s
KH_HD uint64_t byte_range_mask(uint32_t lo, uint32_t hi) {
  uint64_t m_hi = hi >= 8 ? ~0ULL : ((1ULL << (8 * hi)) - 1);
  uint64_t m_lo = lo >= 8 ? ~0ULL : ((1ULL << (8 * lo)) - 1);
  return (m_hi & ~m_lo) & 0x8080808080808080ULL;
}
// 8 values at level array a starting at 8-aligned index w8 (past the end reads as 127)
KH_HD uint64_t load8(const uint8_t* a, uint64_t w8, uint64_t sz) {
  if (w8 + 8 <= sz) return *(const uint64_t*)(a + w8);
  uint64_t x = 0x7F7F7F7F7F7F7F7FULL;
  for (uint64_t q = w8; q < sz; ++q) x = (x & ~(0xFFULL << (8 * (q - w8)))) | ((uint64_t)a[q] << (8 * (q - w8)));
  return x;
}
// rightmost index in [lo, hi) of level array a with value < t, or -1
KH_HD int64_t scan_left(const uint8_t* a, uint64_t sz, uint64_t lo, uint64_t hi, uint32_t t) {
  while (hi > lo) {
    uint64_t w8 = (hi - 1) & ~(uint64_t)7;
    uint64_t from = w8 > lo ? w8 : lo;
    uint64_t m = lt_mask(load8(a, w8, sz), t) & byte_range_mask((uint32_t)(from - w8), (uint32_t)(hi - w8));
    if (m) return (int64_t)(w8 + ((63 - clz64(m)) >> 3));
    hi = from;
  }
  return -1;
}
// leftmost index in [lo, hi) with value < t, or -1
KH_HD int64_t scan_right(const uint8_t* a, uint64_t sz, uint64_t lo, uint64_t hi, uint32_t t) {
  while (lo < hi) {
    uint64_t w8 = lo & ~(uint64_t)7;
    uint64_t to = w8 + 8 < hi ? w8 + 8 : hi;
    uint64_t m = lt_mask(load8(a, w8, sz), t) & byte_range_mask((uint32_t)(lo - w8), (uint32_t)(to - w8));
    if (m) return (int64_t)(w8 + (ctz64(m) >> 3));
    lo = to;
  }
  return -1;
}

// largest j < b with u[j] < t; -1 if none (the 64-ary min pyramid bounds each level's
// scan to one 64-entry block).  "<= t" is "< t+1".
KH_HD int64_t ansv_left(const Pyr& P, uint64_t b, uint32_t t) {
  uint64_t pos = b;
  int L = 0;
  int64_t found = -1;
  for (; L < P.nl; ++L) {
    found = scan_left(P.lv[L], P.sz[L], pos & ~(uint64_t)63, pos, t);
    if (found >= 0) break;
    pos >>= 6;
  }
  if (found < 0) return -1;
  for (; L > 0; --L) {
    uint64_t lo = (uint64_t)found * 64;
    uint64_t hi = lo + 64 < P.sz[L - 1] ? lo + 64 : P.sz[L - 1];
    found = scan_left(P.lv[L - 1], P.sz[L - 1], lo, hi, t);
  }
  return found;
}

// smallest j > b with u[j] < t; -1 if none
KH_HD int64_t ansv_right(const Pyr& P, uint64_t b, uint32_t t) {
  uint64_t pos = b;
  int L = 0;
  int64_t found = -1;
  for (; L < P.nl; ++L) {
    uint64_t end = (pos | 63) + 1;
    if (end > P.sz[L]) end = P.sz[L];
    found = scan_right(P.lv[L], P.sz[L], pos + 1, end, t);
    if (found >= 0) break;
    pos >>= 6;
  }
  if (found < 0) return -1;
  for (; L > 0; --L) {
    uint64_t lo = (uint64_t)found * 64;
    uint64_t hi = lo + 64 < P.sz[L - 1] ? lo + 64 : P.sz[L - 1];
    found = scan_right(P.lv[L - 1], P.sz[L - 1], lo, hi, t);
  }
  return found;
}

KH_HD void op_min64(const uint8_t* in, uint64_t nin, uint8_t* out, uint64_t i) {
  uint64_t lo = i * 64, hi = lo + 64 < nin ? lo + 64 : nin;
  uint32_t mn = 255;
  for (uint64_t j = lo; j < hi; ++j) mn = in[j] < mn ? in[j] : mn;
  out[i] = (uint8_t)mn;
}

// Previous smaller-or-equal boundary for every b.  If it carries the same value it is b's
// predecessor in its group (b is not the group's first, and it is not the last); else b
// is its group's representative, and only reps need their strictly-smaller neighbours
// (the range of the branch): psv = pse, nsv one more query.  glast must be preset to 1.
KH_HD void op_ansv(const Topo& T, const Pyr& P, uint64_t b) {
  uint32_t t = T.u[b];
  if (t == 0) {
    T.psv[b] = T.nsv[b] = T.pse[b] = -1;
    return;
  }
  int64_t pse = ansv_left(P, b, t + 1);
  if (pse >= 0 && T.u[pse] == t) {
    T.pse[b] = (int32_t)pse;  // the previous member of b's group
    T.glast[pse] = 0;         // the predecessor has a later member
    return;
  }
  T.pse[b] = -1;  // b is its group's first (the chain walk stops here)
  T.psv[b] = (int32_t)pse;
  T.nsv[b] = (int32_t)ansv_right(P, b, t);
}

// representative flags in bit form (Topo::rep_bits)
KH_HD uint32_t kh_popc(uint32_t x) {
#ifdef __HIP_DEVICE_COMPILE__
  return (uint32_t)__popc(x);
#else
  return (uint32_t)__builtin_popcount(x);
#endif
}
KH_HD void rep_bit_set(const Topo& T, uint64_t b) {
#ifdef __HIP_DEVICE_COMPILE__
  atomicOr(&T.rep_bits[b >> 5], 1u << (b & 31));  // (k_chain_list: after the tile kernel wrote the word)
#else
  T.rep_bits[b >> 5] |= 1u << (b & 31);
#endif
}
// key-order branch id of representative boundary b
KH_HD uint32_t bid_of(const Topo& T, uint64_t b) {
  if (!T.rep_bits) return T.isrep_bid[b];
  const uint64_t w = b >> 5;
  return T.rep_pref[w] + kh_popc(T.rep_bits[w] & ((1u << (b & 31)) - 1u));
}

// ---- stage: group representative and ordinal (walk the PSE chain, <= 14 steps)
KH_HD void op_chain(const Topo& T, uint64_t b) {
  uint32_t t = T.u[b];
  if (t == 0) {
    T.rep[b] = NONE;
    T.ord[b] = 0;
    if (!T.rep_bits) T.isrep_bid[b] = 0;
    return;
  }
  int64_t j = (int64_t)b;
  uint32_t o = 0;
  for (;;) {  // one dependent load per step: pse holds same-group predecessors only
    int32_t q = T.pse[j];
    if (q < 0) break;
    j = q;
    if (++o > 15) {  // impossible for a 16-ary trie: flag corruption
      T.ctr[CTR_ERR] = 1;
      break;
    }
  }
  T.rep[b] = (uint32_t)j;
  T.ord[b] = (uint8_t)o;
  if (!T.rep_bits)
    T.isrep_bid[b] = (o == 0) ? 1u : 0u;
  else if (o == 0)
    rep_bit_set(T, b);
  if (T.glast[b]) T.gk[j] = (uint8_t)(o + 2);  // the group's last member: the branch has o + 2 children
}

// ---- stage: ANSV and chains tile by tile (k_topo_tile).  op_ansv / op_chain above take one
// dependent HBM round trip per pyramid level and per chain step for every boundary.  Here a
// workgroup holds a tile of consecutive boundaries in LDS (with its own 64-ary level) and
// answers every query whose answer lies in the tile.  Listed for op_ansv / op_chain over the
// whole array: the boundaries with no smaller-or-equal one before them in the tile (the tile's
// prefix minima), the representatives whose next strictly smaller boundary lies past it, and
// the members whose chain passes such a boundary or that have no later member in the tile
// while their group's range leaves it.  A link op_ansv makes across tiles always ends at a
// listed boundary, so the global pass sees the same links op_ansv / op_chain would: the
// results are theirs on every boundary (tests/test_emu.py checks it with tiles of 1..4096).
// The tile's two levels (its tn values and the mins of 64 of them) are a fixed-shape TilePyr:
// a Pyr indexed by level would live in scratch memory.
struct TilePyr {
  const uint8_t* l0;
  const uint8_t* l1;
  uint32_t sz0, sz1;
};
// ansv_left / ansv_right over the two levels
KH_HD int64_t tile_left(const TilePyr& P, uint32_t b, uint32_t t) {
  int64_t f = scan_left(P.l0, P.sz0, b & ~63u, b, t);
  if (f >= 0) return f;
  f = scan_left(P.l1, P.sz1, 0, b >> 6, t);
  if (f < 0) return -1;
  const uint32_t lo = (uint32_t)f * 64, hi = lo + 64 < P.sz0 ? lo + 64 : P.sz0;
  return scan_left(P.l0, P.sz0, lo, hi, t);
}
KH_HD int64_t tile_right(const TilePyr& P, uint32_t b, uint32_t t) {
  const uint32_t end = (b | 63u) + 1 < P.sz0 ? (b | 63u) + 1 : P.sz0;
  int64_t f = scan_right(P.l0, P.sz0, b + 1, end, t);
  if (f >= 0) return f;
  f = scan_right(P.l1, P.sz1, (b >> 6) + 1, P.sz1, t);
  if (f < 0) return -1;
  const uint32_t lo = (uint32_t)f * 64, hi = lo + 64 < P.sz0 ? lo + 64 : P.sz0;
  return scan_right(P.l0, P.sz0, lo, hi, t);
}
constexpr uint32_t TOPO_TILE = 4096;
constexpr int16_t LP_OPEN = -2;  // lpse: the link leaves the tile
// phase 1, tile boundary i (global t0 + i): local ANSV; returns true when op_ansv must redo it.
// lnext[j] = 1 marks j as having a later member of its group in the tile (zeroed before the
// phase); lrin[i] = 1 marks a representative whose next strictly smaller boundary is in it.
KH_HD bool op_tile_ansv(const Topo& T, const TilePyr& P, uint64_t t0, uint32_t i, int16_t* lpse, uint8_t* lnext,
                        uint8_t* lrin) {
  const uint64_t b = t0 + i;
  const uint32_t t = P.l0[i];
  if (t == 0) {
    T.psv[b] = T.nsv[b] = T.pse[b] = -1;
    lpse[i] = -1;
    return false;
  }
  const int64_t j = tile_left(P, i, t + 1);  // previous smaller-or-equal in the tile
  if (j < 0) {
    lpse[i] = LP_OPEN;
    return true;
  }
  if (P.l0[j] == t) {  // the previous member of b's group
    lpse[i] = (int16_t)j;
    lnext[j] = 1;
    T.glast[t0 + j] = 0;
    return false;  // (T.pse[b]: phase 2, only where a walk from outside the tile can read it)
  }
  // the group's first member: its range ends at the next strictly smaller boundary
  lpse[i] = -1;
  T.psv[b] = (int32_t)(t0 + j);
  const int64_t q = tile_right(P, i, t);
  if (q < 0) {
    lrin[i] = 0;
    return true;  // beyond the tile
  }
  T.nsv[b] = (int32_t)(t0 + q);
  lrin[i] = 1;
  return false;
}
// phase 2 (after phase 1 on the whole tile): the chain walk over the tile's links; returns true
// when op_chain must redo it: the walk leaves the tile, or b has no later member in the tile
// while its group's range does (it may be the group's last or not).  With T.rep_bits the
// representative flag goes to *isrep (the caller packs the wave's flags into the bit words).
KH_HD bool op_tile_chain(const Topo& T, const TilePyr& P, uint64_t t0, uint32_t i, const int16_t* lpse,
                         const uint8_t* lnext, const uint8_t* lrin, uint32_t* isrep) {
  const uint64_t b = t0 + i;
  if (P.l0[i] == 0) {
    T.rep[b] = NONE;
    T.ord[b] = 0;
    if (!T.rep_bits) T.isrep_bid[b] = 0;
    return false;
  }
  // b's link in global memory (phase 1 left it in LDS): only for groups that leave the tile, whose
  // members op_chain may walk from a listed boundary; a group inside the tile is never walked again
  // (0.4 GB of writes less on the critical path at 100M)
  const int16_t own = lpse[i];
  auto keep_link = [&] {
    if (own != LP_OPEN) T.pse[b] = own < 0 ? -1 : (int32_t)(t0 + (uint32_t)own);
  };
  uint32_t j = i, o = 0;
  for (;;) {
    const int16_t p = lpse[j];
    if (p == LP_OPEN) {
      keep_link();
      return true;
    }
    if (p < 0) break;
    j = (uint32_t)p;
    if (++o > 15) {  // impossible for a 16-ary trie: flag corruption
      T.ctr[CTR_ERR] = 1;
      break;
    }
  }
  const bool last = !lnext[i];
  if (!lrin[j]) keep_link();
  if (last && !lrin[j]) return true;
  T.rep[b] = (uint32_t)(t0 + j);
  T.ord[b] = (uint8_t)o;
  if (T.rep_bits)
    *isrep = o == 0 ? 1u : 0u;
  else
    T.isrep_bid[b] = o == 0 ? 1u : 0u;
  if (last) T.gk[t0 + j] = (uint8_t)(o + 2);  // the group's last member: o + 2 children
  return false;
}

// parent resolution for a node whose key range is [s, e]: boundaries s-1 and e
struct Parent {
  uint32_t bid;  // NONE: top of its segment
  int32_t pd;    // parent depth (depth0-1 for a top)
  uint32_t pord;
};
// Both sides are looked up before the deeper one is chosen: three dependent load rounds
// (boundary value + rep + ordinal of a and c, then the reps' branch ids) instead of four.
KH_HD Parent resolve_parent(const Topo& T, int64_t a, int64_t c) {
  const uint32_t va = a >= 0 ? T.u[a] : 0, vc = c >= 0 ? T.u[c] : 0;
  const uint32_t ra = a >= 0 ? T.rep[a] : NONE, rc = c >= 0 ? T.rep[c] : NONE;
  const uint32_t oa = a >= 0 ? T.ord[a] : 0, oc = c >= 0 ? T.ord[c] : 0;
  uint32_t ba = (va && ra != NONE) ? bid_of(T, ra) : NONE;
  uint32_t bc = (vc && rc != NONE) ? bid_of(T, rc) : NONE;
  if (T.bid_pos) {
    if (ba != NONE) ba = T.bid_pos[ba];
    if (bc != NONE) bc = T.bid_pos[bc];
  }
  Parent P;
  if (va == 0 && vc == 0) {
    P.bid = NONE;
    P.pd = (int32_t)T.depth0 - 1;
    P.pord = 0;
  } else if (va >= vc) {
    P.bid = ba;
    P.pd = (int32_t)va - 1;
    P.pord = oa + 1u;
  } else {
    P.bid = bc;
    P.pd = (int32_t)vc - 1;
    P.pord = oc;
  }
  return P;
}

// ---- stage: branch records (thread per boundary; only reps act).  The child count
// was left by the group's last member (op_chain): its ordinal + 2.
// returns 1 when boundary b made a branch with an extension above it (k_branch_topo's
// extension count: from the values computed here, not a second pass over u, rep and br_ext)
KH_HD uint32_t op_branch_topo(const Topo& T, const Pyr& P, uint64_t nb, uint64_t b) {
  uint32_t j;
  if (T.rep_bits) {  // (the bit words, 12.5 MB at 100M, instead of every boundary's value and rep)
    const uint32_t wd = T.rep_bits[b >> 5], below = wd & ((1u << (b & 31)) - 1u);
    if (!((wd >> (b & 31)) & 1u)) return 0;
    j = T.rep_pref[b >> 5] + kh_popc(below);
  } else {
    if (T.u[b] == 0 || T.rep[b] != (uint32_t)b) return 0;
    j = T.isrep_bid[b];
  }
  uint32_t t = T.u[b];
  if (t > 64 || t < T.depth0 + 1) {  // a corrupt boundary value (see pd_scatter_vals): no depth past the level tables
    T.ctr[CTR_ERR] = ERR_LEAF_TOPO;
    return 0;
  }
  uint32_t d = t - 1u;
  int64_t a = T.psv[b], c = T.nsv[b];
  Parent Pp = resolve_parent(T, a, c);
  T.br_k[j] = T.gk[b];
  T.br_depth[j] = (uint8_t)d;
  T.br_ext[j] = (uint8_t)((int32_t)d - Pp.pd - 1);
  T.br_parent[j] = Pp.bid;
  T.br_pord[j] = (uint8_t)Pp.pord;
  T.br_first[j] = (uint32_t)(a + 1);
  if (T.br_end) T.br_end[j] = c < 0 ? (uint32_t)T.m : (uint32_t)c + 1;  // boundary c follows key c
  return (int32_t)d - Pp.pd - 1 != 0 ? 1u : 0u;
}

// ---- leaf geometry
KH_HD void leaf_value(const Topo& T, uint64_t i, const uint8_t** p, uint64_t* len) {
  *p = T.vals + T.svoff[i];
  *len = T.svlen[i];
}

// gather the value span of sorted key i (random reads once, sequential reads after)
KH_HD void op_val_gather(const Topo& T, uint64_t i) {
  uint32_t src = T.sidx ? T.sidx[i] : (uint32_t)i;  // presorted input: identity
  uint64_t o = T.voff[src];
  T.svoff[i] = o;
  T.svlen[i] = T.vlen_in ? T.vlen_in[src] : (uint32_t)(T.voff[src + 1] - o);
}

// encoded leaf length for path start nibble s (a key of kn nibbles)
KH_HD uint64_t leaf_enc_len(uint32_t s, uint64_t vlen, uint32_t v0, uint32_t kn = 64) {
  uint32_t p = kn - s;
  uint32_t h = p / 2 + 1;                   // HP bytes; first byte 0x2_/0x3_ < 0x80
  uint64_t hp = h == 1 ? 1 : 1 + h;         // h <= 33 < 56
  uint64_t payload = hp + rlp_str_len(vlen, v0);
  return rlp_hdr_len(payload) + payload;
}

// alloc(bytes) -> offset in the long-leaf region (device: an atomic bump on
// CTR_LFBYTES; long leaves are rare, so there is no contention)
template <typename AllocFn>
KH_HD void op_leaf_topo(const Topo& T, uint64_t i, AllocFn alloc) {
  int64_t a = (int64_t)i - 1, c = (i + 1 < T.m) ? (int64_t)i : -1;
  Parent P = resolve_parent(T, a, c);
  T.lf_parent[i] = P.bid;
  T.lf_pord[i] = (uint8_t)P.pord;
  T.lf_pd[i] = (int8_t)P.pd;
  if (el_cached(T, i, (uint32_t)(P.pd + 1))) {
    T.lf_aoff[i] = 0;
    T.lf_len[i] = T.el_crl[i];
    return;
  }
  if (el_subtree(T, i)) {
    const uint32_t e = el_ext_nibbles(T, i, (uint32_t)(P.pd + 1));
    T.lf_aoff[i] = 0;
    T.lf_len[i] = e ? ext_enc_len(e, T.el_brl[i]) : T.el_brl[i];
    return;
  }
  if (is_branch_value(T, i)) {  // no node: the parent branch holds the value
    T.lf_aoff[i] = 0;
    T.lf_len[i] = 0;
    return;
  }
  const uint8_t* vp;
  uint64_t vlen;
  leaf_value(T, i, &vp, &vlen);
  uint32_t v0 = vlen == 1 ? (uint32_t)*vp : 0;  // the first byte matters only for a 1-byte value
  uint64_t L = leaf_enc_len((uint32_t)(P.pd + 1), vlen, v0, key_nibs(T, i));
  T.lf_aoff[i] = L > LEAF_SHORT_MAX ? alloc((L + 7) & ~(uint64_t)7) : 0;
}

// ---- node hashing is split in two kernels per node set:
//   prep: RLP-encode the node into its arena slot (memory-bound, many waves in
//         flight to hide the gathers of values / child references),
//   hash: Keccak-256 of the arena bytes (aligned, independent loads; VALU-bound)
// and the hash step publishes the node's reference into its parent's child record.

// ---- publishing a finished node's reference into its parent's child record or
// the segment result.  enc: the node's encoding in the arena (used when L < 32).
constexpr uint16_t CM_BR = 0x4000;  // leaf positions: the record is a branch child's (cend holds its end)
KH_HD void publish_ref(const Topo& T, uint32_t parent, uint32_t pord, uint32_t nib, uint64_t first_key,
                       const uint64_t* enc, uint32_t L, const uint64_t h[4], uint16_t mflag = 0) {
  uint64_t w[4];
  for (int j = 0; j < 4; ++j) {
    uint32_t base = 8u * (uint32_t)j;
    w[j] = L >= 32 ? h[j] : (base < L ? (enc[j] & low_bytes_mask(L - base < 8 ? L - base : 8)) : 0);
  }
  if (parent == NONE) {
    uint32_t r = result_index(T, first_key);
    for (int j = 0; j < 4; ++j) {
      T.res_hash[4 * r + j] = h[j];
      T.res_inl[4 * r + j] = L < 32 ? w[j] : 0;
    }
    T.res_len[r] = L;
  } else {
    uint64_t slot = (uint64_t)T.br_cbase[parent] + pord;
    for (int j = 0; j < 4; ++j) T.cref[4 * slot + j] = w[j];
    T.cmeta[slot] = (uint16_t)((L >= 32 ? 32u : L) | (nib << 8) | mflag);
  }
}

// Keccak-256 of an arena message, skipped for an inline (< 32 B) non-top node: the
// reference never hashes a node it embeds.  Returns permutations spent.
KH_HD uint32_t hash_node(const uint64_t* enc, uint32_t L, bool top, uint64_t h[4]) {
  if (L < 32 && !top) {
    h[0] = h[1] = h[2] = h[3] = 0;
    return 0;
  }
  kec256_msg<true>((const uint8_t*)enc, L, h);
  return perms_for_len(L);
}
KH_HD void kec256_strided(const uint64_t* w, uint64_t stride, uint32_t len, uint64_t out[4]);
KH_HD uint32_t hash_slot(const Slot& sl, uint32_t L, bool top, uint64_t h[4]) {
  if (L < 32 && !top) {
    h[0] = h[1] = h[2] = h[3] = 0;
    return 0;
  }
  kec256_strided(sl.w, sl.stride, L, h);
  return perms_for_len(L);
}
KH_HD void slot_head(const Slot& sl, uint32_t L, uint64_t head[4]) {
  for (int q = 0; q < 4; ++q) head[q] = (8u * q < L) ? sl.w[q * sl.stride] : 0;
}

template <typename W>
KH_HD void bw_ref(W& w, const uint64_t r[4], uint32_t len) {  // child reference: 0xa0+hash or inline bytes
  if (len == 32) {
    w.put1(0xA0);
    w.put(r[0], 8);
    w.put(r[1], 8);
    w.put(r[2], 8);
    w.put(r[3], 8);
  } else {
    w.words(r, len);
  }
}

// ---- leaf prep: [HP(path, leaf), value] into the message store (thread per leaf)
// Leaf encoding RLP[HP(path, leaf), value] (MerklePatriciaTrie.scala:565-583):
// a header of P = L - vlen bytes (list prefix, HP prefix, key suffix, value prefix)
// followed by the value bytes.
struct LeafGeom {
  uint32_t s;        // first path nibble (parent depth + 1)
  uint32_t h;        // HP bytes
  uint32_t hp0;      // first HP byte
  uint64_t payload;  // list payload length
  uint32_t L;        // encoding length
  uint32_t v0;       // the value's first byte (only read for a 1-byte value)
  uint32_t kb;       // key bytes (32; fewer for variable-length keys)
};
KH_HD LeafGeom leaf_geom(const Key4& k, int32_t pd, uint64_t vlen, uint32_t v0, uint32_t kn = 64) {
  LeafGeom g;
  g.s = (uint32_t)(pd + 1);
  g.kb = kn / 2;
  uint32_t p = kn - g.s;
  g.h = p / 2 + 1;
  g.hp0 = (p & 1) ? (0x30u | key_nibble(k, (int)g.s)) : 0x20u;
  uint64_t hpl = g.h == 1 ? 1 : 1 + g.h;
  g.payload = hpl + rlp_str_len(vlen, v0);
  g.L = (uint32_t)(rlp_hdr_len(g.payload) + g.payload);
  g.v0 = v0;
  return g;
}
KH_HD void leaf_header(BW& w, const Key4& k, const LeafGeom& g, uint64_t vlen) {
  w.len_prefix(g.payload, 0xC0);
  if (g.h > 1) w.put1(0x80 + g.h);
  w.put1(g.hp0);
  w.key_suffix(k, (g.s + 1) / 2, g.kb);
  if (!(vlen == 1 && g.v0 < 0x80)) w.len_prefix(vlen, 0x80);
}

// vp: the value bytes (global memory, or a staged copy in LDS on the device)
KH_HD void op_leaf_prep(const Topo& T, uint64_t i, const uint8_t* vp, uint64_t vlen) {
  const Key4 k = sorted_key(T, i, 64);
  if (el_cached(T, i, (uint32_t)(T.lf_pd[i] + 1))) return;
  if (el_subtree(T, i)) {  // extension over the unchanged branch (nothing when it hangs at its own depth)
    const uint32_t a = (uint32_t)(T.lf_pd[i] + 1), e = el_ext_nibbles(T, i, a);
    if (!e) return;
    const uint32_t brl = T.el_brl[i], hl = e / 2 + 1;
    const uint32_t xpay = (hl == 1 ? 1 : 1 + hl) + (brl >= 32 ? 33 : brl);
    BW x(T.lmsg + i, T.lstride);
    x.len_prefix(xpay, 0xC0);
    if (hl > 1) x.put1(0x80 + hl);
    uint32_t q = a;
    if (e & 1) {
      x.put1(0x10u | key_nibble(k, (int)q));
      ++q;
    } else {
      x.put1(0x00);
    }
    for (; q < T.el_db[i]; q += 2) x.put1((key_nibble(k, (int)q) << 4) | key_nibble(k, (int)q + 1));
    bw_ref(x, T.el_bref + 4 * i, brl >= 32 ? 32 : brl);
    x.flush();
    return;
  }
  if (is_branch_value(T, i)) return;
  uint32_t v0 = vlen == 1 ? (uint32_t)*vp : 0;  // the first byte matters only for a 1-byte value
  LeafGeom g = leaf_geom(k, T.lf_pd[i], vlen, v0, key_nibs(T, i));
  BW w = g.L <= LEAF_SHORT_MAX ? BW(T.lmsg + i, T.lstride) : BW((uint64_t*)(T.arena + T.lf_aoff[i]), 1);
  leaf_header(w, k, g, vlen);
  w.bytes(vp, vlen);
  w.flush();
  T.lf_len[i] = g.L;
}

// Keccak-256 of a message whose words are `stride` words apart (any length)
KH_HD void kec256_strided(const uint64_t* w, uint64_t stride, uint32_t len, uint64_t out[4]) {
  KState s = {};
  uint32_t nfull = len / 136;
  for (uint32_t b = 0; b < nfull; ++b) {
#pragma unroll
    for (int q = 0; q < 17; ++q) kxor(s, q, w[q * stride]);
    keccakf(s);
    w += 17 * stride;
  }
  len -= nfull * 136;
#pragma unroll
  for (int q = 0; q < 17; ++q) {
    uint64_t x = 0;
    uint32_t base = 8u * (uint32_t)q;
    if (base < len) x = w[q * stride] & low_bytes_mask(len - base < 8 ? len - base : 8);
    if ((len >> 3) == (uint32_t)q) x ^= 0x01ULL << (8 * (len & 7));
    if (q == 16) x ^= 0x80ULL << 56;
    kxor(s, q, x);
  }
  keccakf(s);
  out[0] = lane(s, 0);
  out[1] = lane(s, 1);
  out[2] = lane(s, 2);
  out[3] = lane(s, 3);
}

// ---- leaf hash (thread per leaf).  Returns permutations spent.
KH_HD uint32_t leaf_nibble(const Topo& T, uint64_t i) {
  const uint32_t pd = (uint32_t)T.lf_pd[i];
  return key_nibble(sorted_key(T, i, pd + 1), (int)pd);
}
// publish of leaf i after hashing: hh = its hash (zero if not hashed: L < 32 and not the
// top), head = its first 4 message words (the inline reference when L < 32)
KH_HD void leaf_publish_at(const Topo& T, uint64_t i, uint32_t L, const uint64_t hh[4], const uint64_t head[4],
                           uint32_t* inl) {
  uint32_t parent = T.lf_parent[i];
  bool top = parent == NONE;
  if (T.lf_hash)
    for (int j = 0; j < 4; ++j) T.lf_hash[4 * i + j] = hh[j];
  if (T.lf_ref) {  // capped reference, for the next incremental commit
    for (int q = 0; q < 4; ++q) {
      uint32_t base = 8u * (uint32_t)q;
      T.lf_ref[4 * i + q] =
          L >= 32 ? hh[q] : (base < L ? head[q] & low_bytes_mask(L - base < 8 ? L - base : 8) : 0);
    }
    T.lf_rlen[i] = L;
  }
  *inl = (L < 32 && !top) ? 1 : 0;
  if (T.cend && !top) {  // leaf positions (a long leaf): the stash, where the parent reads it
    for (int q = 0; q < 4; ++q) {
      uint32_t base = 8u * (uint32_t)q;
      T.lf_eref[4 * i + q] = L >= 32 ? hh[q] : (base < L ? head[q] & low_bytes_mask(L - base < 8 ? L - base : 8) : 0);
    }
    T.lf_emeta[i] = (uint8_t)(L >= 32 ? 32 : L);
    return;
  }
  uint32_t nib = top ? 0 : leaf_nibble(T, i);
  publish_ref(T, parent, T.lf_pord[i], nib, i, head, L, hh);
}

// hash + publish of leaf i whose encoding (L bytes) sits at w, words `stride` apart
KH_HD uint32_t leaf_hash_at(const Topo& T, uint64_t i, const uint64_t* w, uint64_t stride, uint32_t L,
                            uint32_t* inl) {
  bool top = T.lf_parent[i] == NONE;
  uint64_t hh[4] = {0, 0, 0, 0}, head[4];
  uint32_t perms = 0;
  if (L <= LEAF_SHORT_MAX) {
    if (L >= 32 || top) {
      kec256_strided(w, stride, L, hh);
      perms = 1;
    }
    for (int q = 0; q < 4; ++q) head[q] = (8u * q < L) ? w[q * stride] : 0;
  } else {
    perms = hash_node(w, L, top, hh);
    for (int q = 0; q < 4; ++q) head[q] = w[q];
  }
  leaf_publish_at(T, i, L, hh, head, inl);
  return perms;
}

KH_HD uint32_t op_leaf_hash(const Topo& T, uint64_t i, uint32_t* inl) {
  *inl = 0;
  if (is_branch_value(T, i)) {  // the value's place in the parent's child records
    const uint64_t slot = (uint64_t)T.br_cbase[T.lf_parent[i]] + T.lf_pord[i];
    T.cref[4 * slot] = T.svoff[i];
    T.cref[4 * slot + 1] = T.svlen[i];
    T.cref[4 * slot + 2] = T.cref[4 * slot + 3] = 0;
    T.cmeta[slot] = VAL_META;
    return 0;
  }
  uint32_t L = T.lf_len[i];
  const uint32_t a = (uint32_t)(T.lf_pd[i] + 1);
  const bool cached = el_cached(T, i, a);
  if (cached || (el_subtree(T, i) && el_ext_nibbles(T, i, a) == 0)) {
    // an unchanged node at its old anchor, or a branch hanging at its own depth: its capped
    // reference goes to the parent; as a top node (the root) it is always hashed, also when
    // its encoding (then held inline) is < 32 B
    const uint64_t* r = cached ? T.el_cref + 4 * i : T.el_bref + 4 * i;
    uint64_t hh[4] = {r[0], r[1], r[2], r[3]}, head[4] = {r[0], r[1], r[2], r[3]};
    uint32_t perms = 0;
    if (L < 32 && T.lf_parent[i] == NONE) {
      kec256_msg<false>((const uint8_t*)head, L, hh);
      perms = 1;
    }
    leaf_publish_at(T, i, L, hh, head, inl);
    *inl = 0;  // embedded or referenced, it is not a node of this build
    return perms;
  }
  if (L <= LEAF_SHORT_MAX) return leaf_hash_at(T, i, T.lmsg + i, T.lstride, L, inl);
  return leaf_hash_at(T, i, (const uint64_t*)(T.arena + T.lf_aoff[i]), 1, L, inl);
}

// ---- early leaves: parent depth from the two adjacent boundaries (= resolve_parent's pd)
constexpr uint8_t EMETA_LONG = 0xFF;
constexpr uint64_t PDINV_SKIP = ~0ULL;
// Plain root builds hash their leaves in INPUT order right after op_lcp, on a second
// stream, while the branch topology is computed.  Input order reads the keys and the
// packed values sequentially (the sorted order would gather every value span at random:
// ~2.5x the algorithmic bytes through 128-byte lines).  op_pd_scatter hands each kept
// input its parent depth (from its sorted neighbours' boundaries) and its sorted
// position, where the leaf kernel stashes the reference (one scattered 33-byte write,
// fire-and-forget); op_leaf_topo_early then moves it into the parent's child record.
KH_HD void op_pd_scatter(const Topo& T, uint64_t i) {
  pd_scatter_vals(T, i, i > 0 ? T.u[i - 1] : 0, i + 1 < T.m ? T.u[i] : 0);
}
// ---- leaf message assembly on 32-bit dwords (k_leaf_in).  The message of a short
// account leaf is prefix [0, o1) | key bytes [kb0, 32) at [o1, e) | value prefix [e, P) |
// value [P, L) (leaf_header's bytes).  The key and the value are loaded at addresses
// shifted by their message position (a second, dependent round trip: the loads then land
// one byte funnel away from their message dwords), so every message dword is one v_perm_b32
// of two loaded dwords, plus byte masks only where a boundary (e, P, L) can fall.  Which
// dwords can hold a boundary is decided per WAVE: the wave's min/max of e and L (DPP
// reductions on the device) make every other dword a single perm, chosen by a scalar
// branch.  WAVE(use, e, Llo, Lhi) returns bounds containing every using lane's values; the
// host replay (tests/emu) passes both the loosest bounds (every dword masked) and the
// lane's own (every dword classified), so both forms are checked against the oracle.
struct WaveBounds {
  uint32_t emin, emax, Lmin, Lmax;
};
// v_perm_b32 with selectors 0..7 (bytes of {hi:lo})
KH_HD uint32_t perm_b32(uint32_t hi, uint32_t lo, uint32_t sel) {
#ifdef __HIP_DEVICE_COMPILE__
  return __builtin_amdgcn_perm(hi, lo, sel);
#else
  const uint64_t d = ((uint64_t)hi << 32) | lo;
  uint32_t r = 0;
  for (int i = 0; i < 4; ++i) r |= (uint32_t)((d >> (8 * ((sel >> (8 * i)) & 7))) & 0xFF) << (8 * i);
  return r;
#endif
}
// bytes below bit position y8 (= 8 x byte count, any int): 0 for y8 <= 0, ~0 for y8 >= 32
KH_HD uint32_t below_mask(int32_t y8) {
  const int32_t c = y8 < 0 ? 0 : y8 > 32 ? 32 : y8;
  return (uint32_t)((0xFFFFFFFFull << c) >> 32);
}
#ifdef __HIP_DEVICE_COMPILE__
#define KH_NOSPEC() asm volatile("")  // not speculated: the enclosing branch stays a branch
#else
#define KH_NOSPEC() ((void)0)
#endif
// A copy of x the compiler cannot see through: table addresses computed from it are neither
// CSE'd with nor hoisted above earlier ones.  k_branch_fused sits at its VGPR limit; without
// this the five 64-bit addresses of its branch's own table entries (br_first, br_end, br_ext,
// br_parent, br_depth at j), formed at entry, stayed live across the permutations for the
// publish and were spilled to scratch (10 VGPRs, 16 scratch instructions a thread).
KH_HD uint32_t opaque_u32(uint32_t x) {
#ifdef __HIP_DEVICE_COMPILE__
  asm volatile("" : "+v"(x));
#endif
  return x;
}
// 4 / 16 bytes from a 4-byte-aligned global address
#ifdef __HIP_DEVICE_COMPILE__
typedef uint32_t v4u_a4 __attribute__((ext_vector_type(4), aligned(4)));
KH_HD uint32_t ld32_a4(uintptr_t a) { return *(const __attribute__((address_space(1))) uint32_t*)a; }
KH_HD void ld128_a4(uintptr_t a, uint32_t* o) {  // global_load_dwordx4 (gfx950 allows 4-byte alignment)
  const v4u_a4 x = *(const __attribute__((address_space(1))) v4u_a4*)a;
  o[0] = x.x;
  o[1] = x.y;
  o[2] = x.z;
  o[3] = x.w;
}
#else
KH_HD uint32_t ld32_a4(uintptr_t a) {
  uint32_t x;
  memcpy(&x, (const void*)a, 4);
  return x;
}
KH_HD void ld128_a4(uintptr_t a, uint32_t* o) { memcpy(o, (const void*)a, 16); }
#endif
constexpr uint32_t LEAF_VD = 36;  // value dwords loaded per lane (the message's 34 + funnel)
constexpr uint32_t LEAF_KD = 12;  // key dwords (message dwords 0..9 + funnel)

// The straight-line permutation of the leaf kernel placed at a fixed offset from a 64-byte
// boundary: KH_LEAF_PAD 4-byte s_nops after a .p2align 6 (measurement builds: -DKH_LEAF_PAD=k;
// unset: no alignment)
#if defined(__HIP_DEVICE_COMPILE__) && defined(KH_LEAF_PAD)
#define KH_STR2(x) #x
#define KH_STR(x) KH_STR2(x)
#define KH_LEAF_ALIGN() asm volatile(".p2align 6\n\t.rept " KH_STR(KH_LEAF_PAD) "\n\ts_nop 0\n\t.endr")
#else
#define KH_LEAF_ALIGN() ((void)0)
#endif
KH_HD uint32_t rlp_hdr_len32(uint32_t x) {  // rlp_hdr_len of a 32-bit length
  return x < 56 ? 1u : x < 0x100u ? 2u : x < 0x10000u ? 3u : x < 0x1000000u ? 4u : 5u;
}
// One leaf: input j (key kin[j], value vals[off .. off + vlen) = voff[j]..voff[j+1]) with
// parent depth pd, stashed at sorted position si.  live = false: a lane that only takes part
// in the wave reductions.  vend: the end of the value buffer, vals + voff[n] (the caller reads
// it once: a load inside the kernel's loop would be one more dependent round trip per input).
template <typename WAVE>
KH_HD uint32_t op_leaf_core(const Topo& T, bool live, int32_t pd, uint32_t si, uint64_t j, uint64_t n, uint64_t off,
                            uint32_t vlen, uintptr_t vend, WAVE wave, uint32_t* inl, uint32_t* longb) {
  *inl = 0;
  *longb = 0;
  if (!live) {
    pd = 0;
    off = 0;
    vlen = 0;
  }
  // geometry (leaf_geom / leaf_header), 32-bit.  A 1-byte value < 0x80 is its own encoding
  // (no prefix): that only shortens L by one and never changes the list-prefix length
  // (the payload stays < 56), so everything up to P is known before the value is read.
  const uint32_t s = (uint32_t)(pd + 1), p = 64 - s, h = p / 2 + 1, hpl = h == 1 ? 1 : 1 + h;
  const uint32_t vhl = rlp_hdr_len32(vlen);
  const uint32_t pay = hpl + vhl + vlen;
  const uint32_t lhl = rlp_hdr_len32(pay);  // 1 or 2 for a short leaf; exact for the long ones
  const uint32_t Lnr = lhl + pay;  // L unless the value is a raw single byte
  const bool lng = Lnr > LEAF_SHORT_MAX;
  const bool use = live && !lng;
  const uint32_t o1 = lhl + (h > 1 ? 1 : 0) + 1, kb0 = (s + 1) >> 1, e = o1 + 32 - kb0, P = e + vhl;
  const WaveBounds B = wave(use, e, vlen == 1 ? e + 1 : Lnr, Lnr);
  if (live && lng) {  // encoded + hashed by op_leaf_long into its arena slot
    T.lf_emeta[si] = EMETA_LONG;
    *longb = (Lnr + 7) & ~7u;
    if (T.longlist) T.longlist[ctr_add(&T.ctr[CTR_LONGN], 1)] = si;  // leaf positions: the post-join pass finds it
  }
  if (!use) return 0;
  // ---- second round trip: the value's first byte, the key and the value at their shifts
  const uint32_t v0 = vlen == 1 ? (uint32_t)T.vals[off] : 0;
  const bool raw = vlen == 1 && v0 < 0x80;
  const uint32_t L = raw ? e + 1 : Lnr;
  uint32_t KD[LEAF_KD], VD[LEAF_VD];
  {  // message byte x <- key byte x + kd  (x in [o1, e))
    const uintptr_t kb = (uintptr_t)(T.kin + 4 * j);
    const int32_t kd = (int32_t)kb0 - (int32_t)o1;
    const int32_t kd0 = kd >> 2;
    if (j == 0 || j + 3 > n) {  // the shifted window would leave the key buffer: clamped dwords
#pragma unroll
      for (uint32_t i = 0; i < LEAF_KD; ++i) {
        const int32_t q = kd0 + (int32_t)i;
        KD[i] = ld32_a4(kb + 4 * (uint32_t)(q < 0 ? 0 : q > 7 ? 7 : q));
      }
    } else {
#pragma unroll
      for (uint32_t g = 0; g < LEAF_KD / 4; ++g) ld128_a4(kb + (intptr_t)4 * kd0 + 16 * g, KD + 4 * g);
    }
  }
  const uintptr_t VB = (uintptr_t)(T.vals + off) - P;  // address of message byte 0 in value space
  const uintptr_t VBa = VB & ~(uintptr_t)3;
  {
    const uintptr_t lo4 = (uintptr_t)T.vals & ~(uintptr_t)3;
    const uintptr_t hi4 = (vend + 3) & ~(uintptr_t)3;
    if (VBa < lo4 || VBa + 4 * LEAF_VD > hi4) {  // the window leaves the value buffer: dword by dword
#pragma unroll
      for (uint32_t i = 0; i < LEAF_VD; ++i) {
        const uintptr_t a = VBa + 4 * i;
        VD[i] = (a >= lo4 && a < hi4) ? ld32_a4(a) : 0;
      }
    } else {
#pragma unroll
      for (uint32_t g = 0; g < LEAF_VD / 4; ++g) ld128_a4(VBa + 16 * g, VD + 4 * g);
    }
  }
  // ---- assembly
  const uint32_t ksel = 0x03020100u + (uint32_t)(((int32_t)kb0 - (int32_t)o1) & 3) * 0x01010101u;
  const uint32_t vsel = 0x03020100u + (uint32_t)(VB & 3) * 0x01010101u;
  const int32_t E8 = 8 * (int32_t)e, P8 = 8 * (int32_t)P, L8 = 8 * (int32_t)L, O8 = 8 * (int32_t)o1;
  const uint32_t vh = raw ? v0 : vlen < 56 ? 0x80 + vlen : (0xB8u | (vlen << 8));  // bytes [e, P) (raw: [e, L))
  const uint64_t vhw = (uint64_t)vh << (8 * (e & 3));
  const uint32_t me = e >> 2, mL = L >> 2, pb = 1u << (8 * (L & 3));
  const uint32_t payl = L - lhl;
  uint32_t pre = lhl == 1 ? 0xC0u + payl : (0xF8u | (payl << 8));  // bytes [0, o1)
  if (h > 1) pre |= (0x80u + h) << (8 * lhl);
  pre |= ((p & 1) ? 0x30u : 0x20u) << (8 * (o1 - 1));
  const uint32_t k0keep = (p & 1) ? 0x0Fu << (8 * (o1 - 1)) : 0;  // the first path nibble rides in the HP byte
  KState S;
#pragma unroll
  for (int m = 0; m < 34; ++m) {
    const uint32_t b0 = 4u * (uint32_t)m;
    // (the conditions are wave-uniform: KH_NOSPEC keeps each masked form behind its scalar
    // branch instead of letting the compiler compute every mask and select)
    uint32_t x = 0;
    if (m <= 9 && b0 < B.emax) {  // key bytes can be here
      uint32_t k = perm_b32(KD[m + 1], KD[m], ksel);
      if (m == 0) {
        k &= (below_mask(E8) & ~below_mask(O8)) | k0keep;
      } else if (b0 + 4 > B.emin) {
        KH_NOSPEC();
        k &= below_mask(E8 - 32 * m);
      }
      x = k;
    }
    if (b0 + 4 > B.emin + 1 && b0 < B.Lmax) {  // value bytes can be here (P >= e + 1, P <= e + 2)
      uint32_t v = perm_b32(VD[m + 1], VD[m], vsel);
      if (b0 < B.emax + 2) {
        KH_NOSPEC();
        v &= ~below_mask(P8 - 32 * m);
      }
      if (b0 + 4 > B.Lmin) {
        KH_NOSPEC();
        v &= below_mask(L8 - 32 * m);
      }
      x |= v;
    }
    if (b0 + 4 > B.emin && b0 <= B.emax + 1) {  // the value prefix can be here
      KH_NOSPEC();
      x |= (uint32_t)m == me ? (uint32_t)vhw : (uint32_t)m == me + 1 ? (uint32_t)(vhw >> 32) : 0u;
    }
    if (m == 0) x |= pre;
    if (b0 + 4 > B.Lmin && b0 <= B.Lmax) {  // padding (KeccakCore.scala:537-546)
      KH_NOSPEC();
      x ^= (uint32_t)m == mL ? pb : 0u;
    }
    if (m == 33) x ^= 0x80u << 24;
    if (m & 1)
      S.hi[m >> 1] = x;
    else
      S.lo[m >> 1] = x;
  }
#pragma unroll
  for (int q = 17; q < 25; ++q) S.lo[q] = S.hi[q] = 0;
  const bool top = pd == (int32_t)T.depth0 - 1;
  uint64_t* r = T.lf_eref + 4 * si;
  uint32_t perms = 0;
  if (L >= 32 || top) {  // a leaf embedded in its parent is never hashed (Node.scala:114)
    KH_LEAF_ALIGN();
    keccakf<KECCAK_FULL>(S);
    for (int q = 0; q < 4; ++q) r[q] = lane(S, q);
    perms = 1;
  } else {  // the encoding itself: the message words without the padding byte at L (< 32);
            // rebuilt here rather than kept live across the permutation (VGPRs)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const uint32_t lo = S.lo[q] ^ ((uint32_t)(2 * q) == mL ? pb : 0u);
      const uint32_t hi = S.hi[q] ^ ((uint32_t)(2 * q + 1) == mL ? pb : 0u);
      r[q] = ((uint64_t)hi << 32) | lo;
    }
    *inl = 1;
  }
  // a top leaf is >= 35 B, so its stash is always the hash; the preset 32 stands for every
  // hashed leaf (one scattered byte write less per leaf)
  if (L < 32) T.lf_emeta[si] = (uint8_t)L;
  // leaf positions: a top leaf (a trie or subtrie of one key) is published after the join by
  // k_leaf_fix, with the long leaves (op_leaf_topo_early publishes a top leaf's stash)
  if (top && T.longlist) T.longlist[ctr_add(&T.ctr[CTR_LONGN], 1)] = si;
  return perms;
}
// input order (the emulator's replay of k_leaf_in, which prefetches pdinv/voff itself): the
// parent depth and sorted position scattered by k_ansv_pd
template <typename WAVE>
KH_HD uint32_t op_leaf_in3(const Topo& T, uint64_t j, uint64_t n, WAVE wave, uint32_t* inl, uint32_t* longb) {
  const uint64_t pv = j < n ? T.pdinv[j] : PDINV_SKIP;
  const bool live = pv != PDINV_SKIP;  // not an earlier put of a key put again later
  const uint64_t off = live ? T.voff[j] : 0;
  const uint32_t vlen = live ? (uint32_t)(T.voff[j + 1] - off) : 0;
  return op_leaf_core(T, live, (int32_t)(int8_t)(uint8_t)(pv >> 32), (uint32_t)pv, j, n, off, vlen,
                      (uintptr_t)T.vals + T.voff[n], wave, inl, longb);
}
// value span of sorted leaf i (early builds gather no spans: through the input index)
KH_HD void leaf_span_early(const Topo& T, uint64_t i, uint64_t* off, uint32_t* len) {
  if (T.svoff) {
    *off = T.svoff[i];
    *len = T.svlen[i];
    return;
  }
  const uint32_t j = T.sidx ? T.sidx[i] : (uint32_t)i;
  *off = T.voff[j];
  *len = (uint32_t)(T.voff[j + 1] - *off);
}
// The early leaves' publish in two halves.  op_leaf_link runs on the topology stream
// right after the branch topology, while the leaves are still being hashed on the other
// stream: sorted leaf i's parent (resolve_parent), child-record slot and nibble.
// op_leaf_move runs after both: the stashed reference is copied to its slot (a streaming
// pass); long and top leaves take op_leaf_topo_early.
constexpr uint64_t LINK_TOP = ~0ULL;
constexpr uint64_t LINK_SLOT = (1ULL << 56) - 1;
KH_HD void op_leaf_link(const Topo& T, uint64_t i) {
  const int64_t a = (int64_t)i - 1, c = (i + 1 < T.m) ? (int64_t)i : -1;
  const Parent P = resolve_parent(T, a, c);
  if (P.bid == NONE) {
    T.lf_dst[i] = LINK_TOP;
    return;
  }
  const Key4 k = sorted_key(T, i, (uint32_t)P.pd + 1);
  T.lf_dst[i] = ((uint64_t)key_nibble(k, P.pd) << 56) | ((uint64_t)T.br_cbase[P.bid] + P.pord);
}
template <typename AllocFn>
KH_HD void op_leaf_topo_early(const Topo& T, uint64_t i, AllocFn alloc);
template <typename AllocFn>
KH_HD void op_leaf_move(const Topo& T, uint64_t i, AllocFn alloc) {
  const uint8_t em = T.lf_emeta[i];
  const uint64_t d = T.lf_dst[i];
  if (em == EMETA_LONG || d == LINK_TOP) {
    op_leaf_topo_early(T, i, alloc);
    return;
  }
  const uint64_t slot = d & LINK_SLOT;
  const uint64_t* r = T.lf_eref + 4 * i;
  const uint64_t r0 = r[0], r1 = r[1], r2 = r[2], r3 = r[3];
  T.cref[4 * slot] = r0;
  T.cref[4 * slot + 1] = r1;
  T.cref[4 * slot + 2] = r2;
  T.cref[4 * slot + 3] = r3;
  T.cmeta[slot] = (uint16_t)(em | ((d >> 56) << 8));
}
// after the branch topology: the stashed reference goes to the parent's child
// record; a long leaf gets its arena slot (as in op_leaf_topo) for op_leaf_long
template <typename AllocFn>
KH_HD void op_leaf_topo_early(const Topo& T, uint64_t i, AllocFn alloc) {
  int64_t a = (int64_t)i - 1, c = (i + 1 < T.m) ? (int64_t)i : -1;
  const uint8_t em = T.lf_emeta[i];
  Parent P = resolve_parent(T, a, c);
  if (em == EMETA_LONG) {
    T.lf_parent[i] = P.bid;
    T.lf_pord[i] = (uint8_t)P.pord;
    T.lf_pd[i] = (int8_t)P.pd;
    uint64_t off;
    uint32_t vlen;
    leaf_span_early(T, i, &off, &vlen);
    uint64_t L = leaf_enc_len((uint32_t)(P.pd + 1), vlen, 0);  // a long value has > 1 byte
    T.lf_aoff[i] = alloc((L + 7) & ~(uint64_t)7);
    return;
  }
  const uint64_t* r = T.lf_eref + 4 * i;
  if (P.bid == NONE) {  // a top leaf: always hashed, its stash is the hash
    publish_ref(T, NONE, 0, 0, i, r, 32, r);
    return;
  }
  const Key4 k = sorted_key(T, i, (uint32_t)P.pd + 1);
  uint64_t slot = (uint64_t)T.br_cbase[P.bid] + P.pord;
  for (int q = 0; q < 4; ++q) T.cref[4 * slot + q] = r[q];
  T.cmeta[slot] = (uint16_t)(em | (key_nibble(k, P.pd) << 8));
}
// a long leaf (> one Keccak block): encode into its arena slot, hash, publish
KH_HD uint32_t op_leaf_long(const Topo& T, uint64_t i, uint32_t* inl) {
  *inl = 0;
  if (T.lf_emeta[i] != EMETA_LONG) return 0;
  uint64_t off;
  uint32_t vlen;
  leaf_span_early(T, i, &off, &vlen);
  op_leaf_prep(T, i, T.vals + off, vlen);
  return leaf_hash_at(T, i, (const uint64_t*)(T.arena + T.lf_aoff[i]), 1, T.lf_len[i], inl);
}

// ---- branch encoding [ref_0 .. ref_15, ""] (Node.scala:31-40): payload length from the
// child records' meta, then the byte stream into any writer (BW: a whole message
// slot; WinBW: one 136-byte Keccak block of it)
KH_HD uint32_t branch_payload(const Topo& T, uint32_t j) {
  uint32_t k = T.br_k[j];
  const uint64_t cb = T.br_cbase[j];
  const uint16_t* cm = T.cmeta + cb;
  uint32_t c0 = 0, term = 1;  // terminator "" (a secure trie never stores a value in a branch)
  if (k && cm[0] == VAL_META) {  // variable-length keys: a key ending here is the 17th item
    const uint64_t vo = T.cref[4 * cb], vl = T.cref[4 * cb + 1];
    term = (uint32_t)rlp_str_len(vl, vl == 1 ? T.vals[vo] : 0);
    c0 = 1;
  }
  uint32_t payload = term + (16 - (k - c0));  // + empty slots
  for (uint32_t c = c0; c < k; ++c) {
    uint32_t len = cm[c] & 0xFF;
    payload += (len == 32) ? 33 : len;
  }
  return payload;
}
template <typename W>
KH_HD void branch_stream(const Topo& T, uint32_t j, W& w, uint32_t payload) {
  uint32_t k = T.br_k[j];
  uint64_t cb = T.br_cbase[j];
  const uint16_t* cm = T.cmeta + cb;
  w.len_prefix(payload, 0xC0);
  const uint64_t* cr = T.cref + 4 * cb;
  const uint32_t c0 = (k && cm[0] == VAL_META) ? 1 : 0;
  int32_t prev = -1;
  for (uint32_t c = c0; c < k; ++c) {
    uint32_t mc = cm[c];
    int32_t nib = (int32_t)(mc >> 8);
    for (int32_t e = prev + 1; e < nib; ++e) w.put1(0x80);  // empty slots
    prev = nib;
    uint64_t r[4] = {cr[4 * c], cr[4 * c + 1], cr[4 * c + 2], cr[4 * c + 3]};
    bw_ref(w, r, mc & 0xFF);
  }
  for (int32_t e = prev + 1; e < 16; ++e) w.put1(0x80);
  if (c0) {  // the value as an RLP string (RLP.scala:141-150)
    const uint64_t vo = cr[0], vl = cr[1];
    const uint8_t* vp = T.vals + vo;
    if (!(vl == 1 && vp[0] < 0x80)) w.len_prefix(vl, 0x80);
    for (uint64_t q = 0; q < vl; ++q) w.put1(vp[q]);
  } else {
    w.put1(0x80);  // terminator (a secure trie never stores a value in a branch)
  }
}

// ---- branch prep: the whole encoding into its message slot (thread per branch of one
// level; g = its position in the level order).  The write-back build keeps it there.
KH_HD void op_branch_prep(const Topo& T, uint32_t j, uint64_t g) {
  uint32_t payload = branch_payload(T, j);
  Slot sl = branch_slot(T, g, T.br_depth[j], false);
  T.br_aoff[j] = g;
  BW w(sl.w, sl.stride);
  branch_stream(T, j, w, payload);
  w.flush();
  T.br_len[j] = rlp_hdr_len(payload) + payload;
}

// Windowed writer: of a byte stream written from position 0, only bytes [w0, w0 + 136)
// (one Keccak block; w0 is a multiple of 136, so 8-aligned) land in the 17-word slot.
struct WinBW {
  BW w;
  uint32_t pos, w0;  // branch encodings are < 600 B
  KH_HD WinBW(uint64_t* d, uint64_t s, uint32_t win0) : w(d, s), pos(0), w0(win0) {}
  KH_HD void put(uint64_t x, uint32_t nb) {
    const uint32_t e = pos + nb;
    if (e > w0 && pos < w0 + 136) {
      if (pos < w0) {
        const uint32_t d = (uint32_t)(w0 - pos);
        x >>= 8 * d;
        nb -= d;
        pos = w0;
      }
      if (pos + nb > w0 + 136) nb = (uint32_t)(w0 + 136 - pos);
      w.put(x, nb);
    }
    pos = e;
  }
  KH_HD void put1(uint32_t b) { put(b, 1); }
  KH_HD void flush() { w.flush(); }
  KH_HD void len_prefix(uint64_t len, uint32_t offset) {
    if (len < 56) {
      put1((uint32_t)(len + offset));
    } else {
      uint32_t nb = be_nbytes(len);
      put1(nb + offset + 55);
      for (int i = (int)nb - 1; i >= 0; --i) put1((uint32_t)(len >> (8 * i)) & 0xFF);
    }
  }
  KH_HD void words(const uint64_t* wd, uint32_t n) {
    for (int j = 0; j < 4 && n; ++j) {
      uint32_t nb = n < 8 ? n : 8;
      put(wd[j], nb);
      n -= nb;
    }
  }
};

// ---- extension (if any) + publish of branch j whose reference is (L, hb, bhead): an
// extension [HP(nibbles pd+1 .. d-1, ext), ref(branch)] is encoded into xs and hashed.
// Returns the permutations spent on the extension; *ninl counts inline nodes.
// where branch j's reference goes: its parent (or the result slot), its nibble there, and
// the extension above it (branch_publish, and k_branch_xl's split form)
struct PubCtx {
  uint32_t ext, parent, d;
  int32_t pd;
  bool top;
  uint64_t first;
  Key4 key;
  uint32_t nib;
  uint16_t mf;
};
KH_HD PubCtx pub_ctx(const Topo& T, uint32_t j) {
  PubCtx P;
  P.ext = T.br_ext[j];
  P.parent = T.br_parent[j];
  P.first = T.br_first[j];
  P.d = T.br_depth[j];
  P.pd = (int32_t)P.d - (int32_t)P.ext - 1;
  P.top = P.parent == NONE;
  P.key = sorted_key(T, P.first, P.d);
  P.nib = P.top ? 0 : key_nibble(P.key, P.pd);
  P.mf = T.cend ? CM_BR : 0;
  return P;
}
// leaf positions: the branch's end position beside its record in the parent
KH_HD void pub_cend(const Topo& T, uint32_t j, const PubCtx& P) {
  if (T.cend && !P.top) T.cend[(uint64_t)T.br_cbase[P.parent] + T.br_pord[j]] = T.br_end[j];
}
// the extension's encoding (HP path + the branch's reference) into xs; its length (T.ex_len)
KH_HD uint32_t ext_encode(const Topo& T, uint32_t j, const PubCtx& P, uint32_t L, const uint64_t hb[4],
                          const uint64_t bhead[4], Slot xs) {
  uint32_t s = (uint32_t)(P.pd + 1);
  uint32_t hl = P.ext / 2 + 1;  // HP bytes
  uint32_t refl = L >= 32 ? 33 : L;
  uint32_t hpl = hl == 1 ? 1 : 1 + hl;  // first HP byte 0x00 / 0x1_ < 0x80
  uint32_t xpay = hpl + refl;
  BW x(xs.w, xs.stride);
  x.len_prefix(xpay, 0xC0);
  if (hl > 1) x.put1(0x80 + hl);
  uint32_t q = s;
  if (P.ext & 1) {
    x.put1(0x10u | key_nibble(P.key, (int)q));
    ++q;
  } else {
    x.put1(0x00);
  }
  for (; q < P.d; q += 2) x.put1((key_nibble(P.key, (int)q) << 4) | key_nibble(P.key, (int)q + 1));
  uint64_t bref[4];
  for (int t = 0; t < 4; ++t) bref[t] = L >= 32 ? hb[t] : bhead[t];
  bw_ref(x, bref, L >= 32 ? 32 : L);
  x.flush();
  uint32_t XL = rlp_hdr_len(xpay) + xpay;
  T.ex_len[j] = XL;
  return XL;
}
// the extension's hash hx (or its inline encoding, read from xs) kept and published
KH_HD void ext_finish(const Topo& T, uint32_t j, const PubCtx& P, uint32_t XL, const uint64_t hx[4], Slot xs,
                      uint32_t* ninl) {
  uint64_t xhead[4];
  slot_head(xs, XL, xhead);
  if (T.ex_hash)
    for (int q2 = 0; q2 < 4; ++q2) T.ex_hash[4 * j + q2] = hx[q2];
  if (T.ex_ref) {
    for (int q2 = 0; q2 < 4; ++q2) {
      uint32_t base = 8u * (uint32_t)q2;
      T.ex_ref[4 * j + q2] =
          XL >= 32 ? hx[q2] : (base < XL ? xhead[q2] & low_bytes_mask(XL - base < 8 ? XL - base : 8) : 0);
    }
    T.ex_rlen[j] = XL;
  }
  *ninl += (XL < 32 && !P.top) ? 1 : 0;
  publish_ref(T, P.parent, T.br_pord[j], P.nib, P.first, xhead, XL, hx, P.mf);
}
KH_HD uint32_t branch_publish(const Topo& T, uint32_t j, uint32_t L, const uint64_t hb[4], const uint64_t bhead[4],
                              Slot xs, uint32_t* ninl) {
  const PubCtx P = pub_ctx(T, j);
  pub_cend(T, j, P);
  if (P.ext == 0) {
    publish_ref(T, P.parent, T.br_pord[j], P.nib, P.first, bhead, L, hb, P.mf);
    return 0;
  }
  const uint32_t XL = ext_encode(T, j, P, L, hb, bhead, xs);
  uint64_t hx[4];
  const uint32_t perms = hash_slot(xs, XL, P.top, hx);
  ext_finish(T, j, P, XL, hx, xs, ninl);
  return perms;
}

// after hashing a branch: per-node hash (write-back) and capped reference (forest records)
KH_HD void branch_keep(const Topo& T, uint32_t j, uint32_t L, const uint64_t hb[4], const uint64_t bhead[4]) {
  if (T.br_hash)
    for (int q = 0; q < 4; ++q) T.br_hash[4 * j + q] = hb[q];
  if (T.br_ref) {
    for (int q = 0; q < 4; ++q) {
      uint32_t base = 8u * (uint32_t)q;
      T.br_ref[4 * j + q] = L >= 32 ? hb[q] : (base < L ? bhead[q] & low_bytes_mask(L - base < 8 ? L - base : 8) : 0);
    }
    T.br_rlen[j] = L;
  }
}

// ---- branch hash (+ extension encode + hash) of a message prepared by op_branch_prep
// (thread per branch of one level; the write-back build)
KH_HD uint32_t op_branch_hash(const Topo& T, uint32_t j, uint64_t g, uint32_t* inl) {
  uint32_t ext = T.br_ext[j];
  uint32_t d = T.br_depth[j];
  bool top = T.br_parent[j] == NONE;
  *inl = 0;
  uint64_t hb[4], bhead[4];
  const uint32_t L = T.br_len[j];
  Slot sl = branch_slot(T, g, d, false);
  uint32_t perms = hash_slot(sl, L, top && ext == 0, hb);
  slot_head(sl, L, bhead);
  uint32_t ninl = (L < 32 && !(top && ext == 0)) ? 1 : 0;
  branch_keep(T, j, L, hb, bhead);
  perms += branch_publish(T, j, L, hb, bhead, branch_slot(T, g, d, true), &ninl);
  *inl = ninl;
  return perms;
}

// ---- fused branch encode + hash (row N1: no node RLP in HBM).  The encoding is streamed
// one 136-byte Keccak block at a time through `slot` (17 words, stride apart: an LDS
// slot of the thread on the device) and absorbed into the state registers as each block
// completes; the child references are read from the contiguous child records.  The
// extension (if any) is encoded into the same slot afterwards.
KH_HD uint32_t op_branch_fused(const Topo& T, uint32_t j, uint64_t* slot, uint64_t stride, uint32_t* inl) {
  uint32_t ext = T.br_ext[j];
  bool top = T.br_parent[j] == NONE;
  *inl = 0;
  uint64_t hb[4] = {0, 0, 0, 0}, bhead[4] = {0, 0, 0, 0};
  uint32_t L, perms = 0, ninl = 0;
  {
    const uint32_t payload = branch_payload(T, j);
    L = rlp_hdr_len(payload) + payload;
    T.br_len[j] = L;
    const bool hashit = L >= 32 || (top && ext == 0);
    const uint32_t nfull = L / 136;
    KState S = {};
    for (uint32_t b = 0; b <= nfull; ++b) {
      WinBW w(slot, stride, 136u * b);
      branch_stream(T, j, w, payload);
      w.flush();
      const uint32_t rem = b < nfull ? 136 : L - 136 * nfull;
      if (!hashit) break;  // embedded in its parent: never hashed (Node.scala:114)
#pragma unroll
      for (int q = 0; q < 17; ++q) {
        const uint32_t base = 8u * (uint32_t)q;
        uint64_t x = base < rem ? slot[q * stride] & low_bytes_mask(rem - base < 8 ? rem - base : 8) : 0;
        if (b == nfull) {
          if ((rem >> 3) == (uint32_t)q) x ^= 0x01ULL << (8 * (rem & 7));
          if (q == 16) x ^= 0x80ULL << 56;
        }
        kxor(S, q, x);
      }
      keccakf(S);
    }
    if (hashit) {
      for (int q = 0; q < 4; ++q) hb[q] = lane(S, q);
      perms = nfull + 1;
    }
    if (L < 32)  // one window: the slot still holds the whole encoding (the inline reference)
      for (int q = 0; q < 4; ++q) {
        const uint32_t base = 8u * (uint32_t)q;
        bhead[q] = base < L ? slot[q * stride] & low_bytes_mask(L - base < 8 ? L - base : 8) : 0;
      }
    ninl = hashit ? 0 : 1;
    branch_keep(T, j, L, hb, bhead);
  }
  perms += branch_publish(T, j, L, hb, bhead, Slot{slot, stride}, &ninl);
  *inl = ninl;
  return perms;
}

// ---- N1 lane variant with direct window assembly (fixed-length keys: no branch values).
// Every empty slot and the terminator of a branch encoding are 0x80, so a 136-byte window
// is prefilled with 0x80 over the encoding's bytes and the list header and each child
// item are XOR-placed at their byte offsets: item c starts at hdr + nibble_c + the running
// sum of (item length - 1) over the children before it.  Per window only the children
// overlapping it are loaded and placed; no byte-serial stream.
KH_HD void window_place(uint64_t* slot, uint64_t stride, uint32_t w0, uint32_t off, uint32_t ilen,
                        const uint64_t I[5]) {
  const uint32_t sh = off & 7, wfirst = off >> 3;
#pragma unroll
  for (uint32_t q = 0; q < 6; ++q) {
    const uint64_t cur = q < 5 ? I[q] : 0, prv = q ? I[q - 1] : 0;
    const uint64_t y = sh ? (cur << (8 * sh)) | (prv >> (64 - 8 * sh)) : cur;
    const uint32_t W = wfirst + q;  // absolute word of the encoding
    const int32_t lo = (int32_t)off - 8 * (int32_t)W, hi = (int32_t)(off + ilen) - 8 * (int32_t)W;
    const uint32_t blo = lo > 0 ? (uint32_t)lo : 0, bhi = hi < 8 ? (hi > 0 ? (uint32_t)hi : 0) : 8;
    if (bhi <= blo || W < w0 / 8 || W >= w0 / 8 + 17) continue;
    const uint64_t m = low_bytes_mask(bhi) & ~low_bytes_mask(blo);
    slot[(W - w0 / 8) * stride] ^= (y ^ 0x8080808080808080ULL) & m;
  }
}
// any active lane of the wave (the host replay: the one lane)
KH_HD bool wave_any(bool p) {
#ifdef __HIP_DEVICE_COMPILE__
  return __ballot(p) != 0;
#else
  return p;
#endif
}
// nibble d of the key at sorted position pos, read as one dword of the input key
KH_HD uint32_t sorted_nibble_deep(const Topo& T, uint64_t pos, uint32_t d) {
  const uint32_t* k = (const uint32_t*)(T.kin + 4 * (uint64_t)T.sidx[pos]);
  const uint32_t b = (k[d >> 3] >> (8 * ((d >> 1) & 3))) & 0xFF;
  return (d & 1) ? b & 0xF : b >> 4;
}
// The same for a hashed child's 33-byte item (0xA0 + hash; the common case), branch-free: it
// covers exactly the 5 words from off / 8; each is funnel-shifted by off % 8 bytes and
// XOR-ed into the window with one LDS atomic (no read-back), a word outside the window
// XOR-ing zero into word 0.
KH_HD void slot_xor(uint64_t* p, uint64_t v) {
#ifdef __HIP_DEVICE_COMPILE__
  __hip_atomic_fetch_xor(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
#else
  *p ^= v;
#endif
}
KH_HD void place33(uint64_t* slot, uint64_t stride, uint32_t w0, uint32_t off, const uint64_t I[5]) {
  const uint32_t sh = off & 7, s = 8 * sh;
  const int32_t r0 = (int32_t)(off >> 3) - (int32_t)(w0 >> 3);
#pragma unroll
  for (uint32_t q = 0; q < 5; ++q) {
    const uint64_t cur = I[q], prv = q ? I[q - 1] : 0;
    const uint64_t y = (cur << s) | ((prv >> 1) >> (63 - s));
    const uint64_t m = q == 0 ? ~0ULL << s : q == 4 ? low_bytes_mask(sh + 1) : ~0ULL;
    const int32_t rel = r0 + (int32_t)q;
    const bool in = rel >= 0 && rel < 17;
    slot_xor(slot + (in ? (uint32_t)rel : 0u) * stride, in ? (y ^ 0x8080808080808080ULL) & m : 0);
  }
}
// Direct window assembly with the children streamed ONCE in order: the window loop
// resumes at the first child not yet placed (an item crossing a window edge is placed
// again, its tail, in the next window), the next child's record is loaded while the
// current one is placed, and the child lengths for the payload are loaded as one batch
// (16 predicated loads issued together).  One Keccak call site (the block loop).
// The child records: by default the level's records in HBM (cm / cr at the branch's child
// base, word q of child c at cr[4c + q]); k_branch_fused<3> (small levels) passes a copy in
// LDS, lane-interleaved: child c's meta at cm[c * cs], word q at cr[(4c + q) * cs].
// leaf positions: the branch kernel reads a leaf child's nibble from the sorted 32-bit
// prefixes (unsegmented: 8 nibbles) for levels below depth 8 (pos_level_ok), and from the
// input key through the sort index below that (SRC_POSK); small levels take their records
// from op_leaf_children
KH_HD bool pos_level_ok(const Topo& T, uint32_t d) { return T.sck && T.ck_sb == 0 && d < 8; }
// the meta of the leaf child at sorted position pos of a branch of the level being built
// (T.lvl_nsh / lvl_depth set for the level: kernel arguments, not registers per lane)
template <bool DEEP>
KH_HD uint32_t leaf_child_meta(const Topo& T, uint64_t pos) {
  const uint32_t len = T.lf_inline ? T.lf_emeta[pos] : 32u;
  const uint32_t nib = DEEP ? key_nibble(sorted_key(T, pos, T.lvl_depth + 1), (int)T.lvl_depth)
                            : (T.sck[pos] >> T.lvl_nsh) & 0xF;
  return len | (nib << 8);
}
// ... and its child records written out (the small levels, whose kernels copy every record
// of a branch at once): the branch's range walked child by child
KH_HD void op_leaf_children(const Topo& T, uint32_t j) {
  const uint32_t k = T.br_k[j], d = T.br_depth[j];
  const uint64_t cb = T.br_cbase[j];
  uint64_t pos = T.br_first[j];
  for (uint32_t c = 0; c < k; ++c) {
    const uint16_t mc = T.cmeta[cb + c];
    if (mc & CM_BR) {
      pos = T.cend[cb + c];
      continue;
    }
    const uint64_t* r = T.lf_eref + 4 * pos;
    for (int q = 0; q < 4; ++q) T.cref[4 * (cb + c) + q] = r[q];
    T.cmeta[cb + c] = (uint16_t)(T.lf_emeta[pos] | (key_nibble(sorted_key(T, pos, d + 1), (int)d) << 8));
    ++pos;
  }
}

struct ChildSrc {
  const uint16_t* cm = nullptr;
  const uint64_t* cr = nullptr;
  uint32_t cs = 1;
  uint32_t* tb = nullptr;  // SRC_T12*: the branch's child table (6 dwords, tbs apart)
  uint32_t tbs = 1;
};
// where op_branch_stream reads the children (one instantiation each, so that a kernel
// carries no dead path: the branch kernels sit at the VGPR limit of 4 waves per SIMD).
// SRC_T12 / SRC_T12K (leaf positions, a branch whose key range is < 4096 positions): every
// child's meta and end are loaded in one round and the leaf children's nibbles in a second,
// and the child loop reads a per-thread table of 12-bit entries (a leaf child's position
// relative to the branch's first key, or a branch child's reference length) from 24 bytes of
// LDS: no dependent metadata load per child, and the table fits beside the window at 4 waves
// per SIMD (16 entries of 32 bits needed 3).
enum { SRC_REC = 0, SRC_LDS = 1, SRC_POS = 3, SRC_POSK = 4, SRC_T12 = 5, SRC_T12K = 6 };
constexpr uint32_t T12_SPAN = 4096;  // key positions a table entry can reach
// PAIR (k_branch_small): lanes 2i and 2i + 1 both run the stream for the same branch (the same
// control flow and stores) and share its permutations, each holding one 32-bit half of every
// state word (keccak.h keccakf_pair); the extension above a branch stays one lane's.
template <int SRC, bool PAIR = false>
KH_HD uint32_t op_branch_stream_t(const Topo& T, uint32_t j, uint64_t* slot, uint64_t stride, uint32_t* inl,
                                  ChildSrc src) {
  const uint32_t ext = T.br_ext[j];
  const bool top = T.br_parent[j] == NONE;
  *inl = 0;
  uint64_t hb[4] = {0, 0, 0, 0}, bhead[4] = {0, 0, 0, 0};
  uint32_t L, perms = 0, ninl = 0;
  {
    const uint32_t k = T.br_k[j];
    // global records are addressed from the branch's child base (one register, not three pointers)
    const uint32_t cb = SRC == SRC_LDS ? 0u : T.br_cbase[j];
    const uint32_t cs = SRC == SRC_LDS ? src.cs : 1u;
    auto cmeta_at = [&](uint32_t c) -> uint32_t { return SRC == SRC_LDS ? src.cm[c * cs] : T.cmeta[cb + c]; };
    auto cref_at = [&](uint32_t c) -> const uint64_t* {
      return SRC == SRC_LDS ? src.cr + 4 * c * cs : T.cref + 4 * (uint64_t)(cb + c);
    };
    uint32_t payload = 1 + (16 - k);  // terminator "" + empty slots
    uint32_t brm = 0;                 // leaf positions: bit c = child c is a branch
    constexpr bool POS = SRC == SRC_POS || SRC == SRC_POSK;
    constexpr bool TBL = SRC == SRC_T12 || SRC == SRC_T12K;
    uint64_t nibs = 0;                                   // TBL: child c's nibble at bits 4c
    const uint32_t kfirst = TBL ? T.br_first[j] : 0u;  // TBL: the positions' origin
    if (TBL) {
      // one round: every child's meta and end (clamped to the last child: no predicated loads;
      // the loops stop at the wave's largest child count)
      uint32_t mc[16], ce[16], lp[16], lm[16];
#pragma unroll
      for (uint32_t c = 0; c < 16; ++c) {
        if (!wave_any(c < k)) break;
        const uint32_t cc = c < k ? c : k - 1;
        mc[c] = T.cmeta[cb + cc];
        ce[c] = T.cend[cb + cc];
      }
      uint32_t pos = kfirst;
#pragma unroll
      for (uint32_t c = 0; c < 16; ++c) {  // the leaf positions (a branch child skips its range)
        if (!wave_any(c < k)) break;
        const bool br = c < k && (mc[c] & CM_BR);
        brm |= br ? 1u << c : 0u;
        lp[c] = pos;
        pos = br ? ce[c] : pos + 1;
      }
      // second round: the leaf children's nibbles (and lengths when a leaf may be inline)
#pragma unroll
      for (uint32_t c = 0; c < 16; ++c) {
        if (!wave_any(c < k)) break;
        const uint32_t p = c < k ? lp[c] : lp[0];
        const uint32_t nib = SRC == SRC_T12K ? sorted_nibble_deep(T, p, T.lvl_depth) : (T.sck[p] >> T.lvl_nsh) & 0xF;
        lm[c] = (T.lf_inline ? T.lf_emeta[p] : 32u) | nib << 8;
      }
      uint32_t tw[6] = {0, 0, 0, 0, 0, 0};
#pragma unroll
      for (uint32_t c = 0; c < 16; ++c) {
        if (!wave_any(c < k)) break;
        const bool br = (brm >> c) & 1;
        const uint32_t m = br ? mc[c] : lm[c];
        const uint32_t len = m & 0xFF;
        if (c < k) {
          payload += len == 32 ? 33 : len;
          nibs |= (uint64_t)((m >> 8) & 0xF) << (4 * c);
        }
        const uint32_t e = (br ? len : lp[c] - kfirst) & 0xFFF;
        const uint32_t bit = 12 * c, d = bit >> 5, sh = bit & 31;
        tw[d] |= e << sh;
        if (sh > 20) tw[d + 1] |= e >> (32 - sh);
      }
#pragma unroll
      for (uint32_t d = 0; d < 6; ++d) src.tb[d * src.tbs] = tw[d];
    } else if (POS) {  // a leaf child's length from its stash meta (32 unless some leaf is inline)
      uint32_t pos = T.br_first[j];
#pragma unroll
      for (uint32_t c = 0; c < 16; ++c) {
        if (c < k) {
          const uint32_t mc = cmeta_at(c);
          const bool br = mc & CM_BR;
          brm |= br ? 1u << c : 0u;
          uint32_t len = br ? mc & 0xFF : 32u;
          if (T.lf_inline) {  // (the positions are walked only when some leaf may be inline)
            if (!br) len = T.lf_emeta[pos];
            pos = br ? T.cend[cb + c] : pos + 1;
          }
          payload += len == 32 ? 33 : len;
        }
      }
    } else {
#pragma unroll
      for (uint32_t c = 0; c < 16; ++c) {
        const uint32_t len = c < k ? (cmeta_at(c) & 0xFF) : 0;
        payload += len == 32 ? 33 : len;
      }
    }
    const uint32_t hh = rlp_hdr_len(payload);
    L = hh + payload;
    T.br_len[j] = L;
    const bool hashit = L >= 32 || (top && ext == 0);
    const uint32_t nfull = L / 136;
    KState S = {};
    auto prefill = [&](uint32_t w0) {  // 0x80 over the encoding's bytes of the window
      if (w0 + 136 <= L) {  // a whole window of the encoding: no masks
#pragma unroll
        for (int q = 0; q < 17; ++q) slot[q * stride] = 0x8080808080808080ULL;
        return;
      }
#pragma unroll
      for (int q = 0; q < 17; ++q) {
        const uint32_t a = w0 + 8u * (uint32_t)q;
        const uint32_t n80 = L > a ? (L - a < 8 ? L - a : 8) : 0;
        slot[q * stride] = low_bytes_mask(n80) & 0x8080808080808080ULL;
      }
    };
    prefill(0);
    {  // the list header
      const uint32_t pl = payload;
      const uint64_t hdr = hh == 1 ? (0xC0 + pl)
                           : hh == 2 ? (0xF8 | ((uint64_t)pl << 8))
                                     : (0xF9 | ((uint64_t)(pl >> 8) << 8) | ((uint64_t)(pl & 0xFF) << 16));
      slot[0] ^= (hdr ^ 0x8080808080808080ULL) & low_bytes_mask(hh);
    }
    // child c's item: I[] and its byte offset / length; the next child's record in flight
    uint32_t c = 0, run = 0, off = 0, ilen = 0;
    uint64_t I[5] = {0, 0, 0, 0, 0};
    uint64_t n0 = 0, n1 = 0, n2 = 0, n3 = 0;
    uint32_t nm = 0;
    uint32_t lpn = POS ? T.br_first[j] : 0;  // leaf positions: sorted position of child cc
    // child c's reference: its record, or (leaf positions) a leaf child's stash at the next
    // position of the range
    auto load_child = [&](uint32_t cc) {
      if (TBL) {  // the table entry: a leaf's position from the branch's first key, a branch child's length
        const uint32_t bit = 12 * cc, d = bit >> 5, sh = bit & 31;
        uint32_t e = src.tb[d * src.tbs] >> sh;
        if (sh > 20) e |= src.tb[(d + 1) * src.tbs] << (32 - sh);
        e &= 0xFFF;
        const bool br = (brm >> cc) & 1;
        const uint32_t len = br ? e : T.lf_inline ? T.lf_emeta[kfirst + e] : 32u;
        nm = len | ((uint32_t)(nibs >> (4 * cc)) & 0xF) << 8;
        const uint64_t* p = br ? T.cref + 4 * (uint64_t)(cb + cc) : T.lf_eref + 4 * (uint64_t)(kfirst + e);
        n0 = p[0], n1 = p[1], n2 = p[2], n3 = p[3];
        return;
      }
      nm = cmeta_at(cc);
      const uint64_t* p = cref_at(cc);
      if (POS) {  // every address known up front (the kind from brm): one round trip
        const bool br = (brm >> cc) & 1;
        const uint32_t lm = leaf_child_meta<SRC == SRC_POSK>(T, lpn), e = T.cend[cb + cc];  // (e: unset for a leaf slot)
        if (!br) p = T.lf_eref + 4 * (uint64_t)lpn;
        nm = br ? nm : lm;
        lpn = br ? e : lpn + 1;
        n0 = p[0], n1 = p[1], n2 = p[2], n3 = p[3];
      } else {
        n0 = p[0], n1 = p[cs], n2 = p[2 * cs], n3 = p[3 * cs];
      }
    };
    if (k) load_child(0);
    bool have = false;  // I / off / ilen hold child c, not yet completely placed
    auto take = [&]() {  // child c from the prefetch registers; prefetch child c + 1
      const uint32_t mc = nm, len = mc & 0xFF;
      ilen = len == 32 ? 33 : len;
      off = hh + ((mc >> 8) & 0xF) + run;
      run += ilen - 1;
      if (len == 32) {
        I[0] = 0xA0 | (n0 << 8);
        I[1] = (n0 >> 56) | (n1 << 8);
        I[2] = (n1 >> 56) | (n2 << 8);
        I[3] = (n2 >> 56) | (n3 << 8);
        I[4] = n3 >> 56;
      } else {  // an embedded child: its bytes (the capped reference is zero past len)
        I[0] = n0;
        I[1] = n1;
        I[2] = n2;
        I[3] = n3;
        I[4] = 0;
      }
      if (c + 1 < k) load_child(c + 1);
      have = true;
    };
    for (uint32_t b = 0; b <= nfull; ++b) {
      const uint32_t w0 = 136u * b;
      if (b) prefill(w0);
      for (;;) {  // place the children overlapping this window, in order
        if (!have) {
          if (c >= k) break;
          take();
        }
        if (off >= w0 + 136) break;  // starts in a later window
        if (ilen == 33)
          place33(slot, stride, w0, off, I);
        else
          window_place(slot, stride, w0, off, ilen, I);
        if (off + ilen > w0 + 136) break;  // its tail goes into the next window too
        have = false;
        ++c;
      }
      if (!hashit) break;  // embedded in its parent: never hashed (Node.scala:114)
      if (b == nfull) {  // the padding, written into the window (two words) rather than
                         // tested for on every word of the absorb
        const uint32_t rem = L - 136 * nfull;
        slot[(rem >> 3) * stride] ^= 0x01ULL << (8 * (rem & 7));
        slot[16 * stride] ^= 0x80ULL << 56;
      }
      if (PAIR) {
        const bool odd = pair_odd();
#pragma unroll
        for (int q = 0; q < 17; ++q) {
          const uint64_t w = slot[q * stride];
          S.lo[q] ^= odd ? (uint32_t)(w >> 32) : (uint32_t)w;
        }
        keccakf_pair(S.lo, odd);
      } else {
#pragma unroll
        for (int q = 0; q < 17; ++q) kxor(S, q, slot[q * stride]);  // zero past the encoding already
        keccakf(S);
      }
    }
    if (hashit) {
      if (PAIR) {
        const bool odd = pair_odd();
        for (int q = 0; q < 4; ++q) {
          const uint32_t m = S.lo[q], o = pair_partner(m);
          hb[q] = odd ? ((uint64_t)m << 32) | o : ((uint64_t)o << 32) | m;
        }
      } else {
        for (int q = 0; q < 4; ++q) hb[q] = lane(S, q);
      }
      perms = nfull + 1;
    }
    if (L < 32)
      for (int q = 0; q < 4; ++q) {
        const uint32_t base = 8u * (uint32_t)q;
        bhead[q] = base < L ? slot[q * stride] & low_bytes_mask(L - base < 8 ? L - base : 8) : 0;
      }
    ninl = hashit ? 0 : 1;
    branch_keep(T, opaque_u32(j), L, hb, bhead);
  }
  perms += branch_publish(T, opaque_u32(j), L, hb, bhead, Slot{slot, stride}, &ninl);
  *inl = ninl;
  return perms;
}

// runtime choice of the child source (the host replay; the kernels instantiate theirs)
KH_HD uint32_t op_branch_stream(const Topo& T, uint32_t j, uint64_t* slot, uint64_t stride, uint32_t* inl,
                                ChildSrc src = ChildSrc{}, bool per_child = false) {
  if (src.cm) return op_branch_stream_t<SRC_LDS>(T, j, slot, stride, inl, src);
  if (T.cend) {
    Topo TL = T;
    TL.lvl_depth = T.br_depth[j];
    TL.lvl_nsh = 28 - 4 * (TL.lvl_depth & 7);
    if (!per_child && T.br_end && T.br_end[j] - T.br_first[j] < T12_SPAN) {  // (per_child: the wide waves' form)
      uint32_t tb[6];
      src.tb = tb;
      src.tbs = 1;
      if (pos_level_ok(T, T.br_depth[j])) return op_branch_stream_t<SRC_T12>(TL, j, slot, stride, inl, src);
      return op_branch_stream_t<SRC_T12K>(TL, j, slot, stride, inl, src);
    }
    if (pos_level_ok(T, T.br_depth[j])) return op_branch_stream_t<SRC_POS>(TL, j, slot, stride, inl, src);
    return op_branch_stream_t<SRC_POSK>(TL, j, slot, stride, inl, src);
  }
  return op_branch_stream_t<SRC_REC>(T, j, slot, stride, inl, src);
}

// node hashes op_branch_hash(T, j, ...) spent `perms` on: the branch if it was
// re-encoded and its encoding is >= 32 B or it is the top; its extension likewise
// (an extension is re-encoded only when perms were spent on it or its branch)
KH_HD uint32_t branch_hash_count(const Topo& T, uint32_t j, uint32_t perms) {
  const bool top = T.br_parent[j] == NONE, ext = T.br_ext[j] != 0;
  uint32_t h = (T.br_len[j] >= 32 || (top && !ext)) ? 1 : 0;
  if (ext && perms) h += (T.ex_len[j] >= 32 || top) ? 1 : 0;
  return h;
}

// Root branch over 16 capped references (the host fold of the sharded path).
// refs: 16 x 4 words, lens: 0 = empty, 32 = hash, else inline length.
// Writes the encoding into out (>= 600 B, 8-aligned); returns its length.
KH_HD uint32_t encode_branch16(const uint64_t* refs, const uint32_t* lens, uint8_t* out) {
  uint32_t payload = 1;
  for (int i = 0; i < 16; ++i) payload += lens[i] == 0 ? 1 : lens[i] == 32 ? 33 : lens[i];
  BW w((uint64_t*)out);
  w.len_prefix(payload, 0xC0);
  for (int i = 0; i < 16; ++i) {
    if (lens[i] == 0) {
      w.put1(0x80);
    } else if (lens[i] == 32) {
      w.put1(0xA0);
      for (int q = 0; q < 4; ++q) w.put(refs[4 * i + q], 8);
    } else {
      w.words(refs + 4 * i, lens[i]);
    }
  }
  w.put1(0x80);
  w.flush();
  return rlp_hdr_len(payload) + payload;
}

}  // namespace khst
