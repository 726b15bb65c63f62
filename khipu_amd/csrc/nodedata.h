// Fast-sync NodeData verification.
//
// NodeDatasRequest.processResponse (sync/package.scala:81-125) hashes every value a
// peer returned, matches the hash against the requested set, decodes a matched trie
// node with PV63's MptNode decoder (PV63.scala:96-127) and lists the child hashes
// still to fetch (getStateNodeChildren / getContractMptNodeChildren,
// sync/package.scala:127-165).  The per-value decode below is shared by the HIP
// kernel and the host replay.  Well-formed nodes decode exactly as the reference;
// malformed input yields a status code where the reference throws.
#pragma once
#include "keccak.h"

namespace khst {

enum NodeKind : uint8_t { NK_STATE = 0, NK_STORAGE_ROOT = 1, NK_CONTRACT = 2, NK_CODE = 3, NK_NONE = 255 };
enum NodeStatus : uint8_t {
  NS_OK = 0,
  NS_NOT_NODE = 1,     // "Cannot decode NodeData"
  NS_BAD_CHILD = 2,    // "unexpected value in node"
  NS_BAD_ACCOUNT = 3,  // "Cannot decode Account" / DataWord / non-value field
  NS_BAD_RLP = 4,      // RLPException: truncated or oversized item, value where a list is needed
};

// One RLP item at d[pos] (RLP.scala getItemBounds, :179-230): payload [off, off+len)
struct RItem {
  uint32_t off, len, next;
  bool list;
};
KH_HD bool rlp_at(const uint8_t* d, uint32_t n, uint32_t pos, RItem& it) {
  if (pos >= n) return false;
  uint32_t p = d[pos];
  uint64_t off, len;
  if (p < 0x80) {
    off = pos;
    len = 1;
    it.list = false;
  } else if (p <= 0xb7) {
    off = pos + 1;
    len = p - 0x80;
    it.list = false;
  } else if (p < 0xc0 || p > 0xf7) {
    uint32_t ll = p < 0xc0 ? p - 0xb7 : p - 0xf7;
    if (ll > 4 || pos + 1 + ll > n) return false;  // "Bytes don't represent an int"
    len = 0;
    for (uint32_t i = 0; i < ll; ++i) len = (len << 8) | d[pos + 1 + i];
    off = pos + 1 + ll;
    it.list = p >= 0xc0;
  } else {
    off = pos + 1;
    len = p - 0xc0;
    it.list = true;
  }
  if (off + len > n) return false;
  it.off = (uint32_t)off;
  it.len = (uint32_t)len;
  it.next = (uint32_t)(off + len);
  return true;
}

// items of a list: fills up to `cap` item records, returns the count (-1 on error)
KH_HD int rlp_items(const uint8_t* d, uint32_t n, const RItem& L, RItem* out, int cap) {
  uint32_t p = L.off, end = L.off + L.len;
  int k = 0;
  while (p < end) {
    RItem it;
    if (!rlp_at(d, n, p, it) || it.next > end) return -1;  // list overrun
    if (k < cap) out[k] = it;
    ++k;
    p = it.next;
  }
  return k;
}

// Canonical re-encoded length of the item at pos (rlp.encode(decoded item)), which
// PV63's decodeChild compares with MaxNodeValueSize; differs from the raw length only
// for non-canonical input.  Bounded recursion (depth <= 16); -1 on error.
KH_HD int64_t rlp_canon_len(const uint8_t* d, uint32_t n, uint32_t pos, int depth) {
  RItem it;
  if (depth > 16 || !rlp_at(d, n, pos, it)) return -1;
  uint64_t pl;
  if (!it.list) {
    if (it.len == 1 && d[it.off] < 0x80) return 1;
    pl = it.len;
  } else {
    pl = 0;
    uint32_t p = it.off, end = it.off + it.len;
    while (p < end) {
      RItem c;
      if (!rlp_at(d, n, p, c) || c.next > end) return -1;
      int64_t cl = rlp_canon_len(d, n, p, depth + 1);
      if (cl < 0) return -1;
      pl += (uint64_t)cl;
      p = c.next;
    }
  }
  uint64_t hdr = 1;
  if (pl >= 56)
    for (uint64_t v = pl; v; v >>= 8) ++hdr;
  return (int64_t)(hdr + pl);
}

// the whole item tree at pos is well formed (rlp.rawDecode decodes it all before
// PV63 looks at it)
KH_HD bool rlp_valid(const uint8_t* d, uint32_t n, uint32_t pos, int depth) {
  RItem it;
  if (depth > 64 || !rlp_at(d, n, pos, it)) return false;
  if (!it.list) return true;
  uint32_t p = it.off, end = it.off + it.len;
  while (p < end) {
    RItem c;
    if (!rlp_at(d, n, p, c) || c.next > end) return false;
    if (c.list && !rlp_valid(d, n, p, depth + 1)) return false;
    p = c.next;
  }
  return true;
}

// PV63 decodeChild for an embedded node: a list of 2 or 17 items whose encoding is
// <= MaxNodeValueSize (31) bytes and that itself decodes as an MptNode.  Checked
// iteratively (an embedded node nests at most a few levels in 31 bytes).
KH_HD uint8_t check_inline_node(const uint8_t* d, uint32_t n, uint32_t pos0) {
  uint32_t stack[16];
  int sp = 0;
  stack[sp++] = pos0;
  while (sp) {
    uint32_t pos = stack[--sp];
    RItem L;
    if (!rlp_at(d, n, pos, L)) return NS_BAD_RLP;
    RItem it[18];
    int k = rlp_items(d, n, L, it, 18);
    if (k < 0) return NS_BAD_RLP;
    if (k == 17) {
      for (int c = 0; c < 16; ++c) {
        if (!it[c].list) {
          if (it[c].len != 32 && it[c].len != 0) return NS_BAD_CHILD;
        } else {
          uint32_t start = c ? it[c - 1].next : L.off;
          RItem sub[18];
          int sk = rlp_items(d, n, it[c], sub, 18);
          if (sk < 0) return NS_BAD_RLP;
          int64_t enc = rlp_canon_len(d, n, start, 0);
          if (!((sk == 2 || sk == 17) && enc >= 0 && enc <= 31)) return NS_BAD_CHILD;
          if (sp >= 16) return NS_BAD_RLP;
          stack[sp++] = start;
        }
      }
      if (it[16].list) return NS_BAD_RLP;  // value slot: byteStringEncDec
    } else if (k == 2) {
      if (it[0].list || it[0].len == 0) return NS_BAD_RLP;  // HexPrefix.decode of a value
      bool leaf = (d[it[0].off] & 0x20) != 0;
      if (leaf) {
        if (it[1].list) return NS_BAD_RLP;  // MptLeaf value: ByteString
      } else if (!it[1].list) {
        if (it[1].len != 32 && it[1].len != 0) return NS_BAD_CHILD;
      } else {
        uint32_t start = it[0].next;
        RItem sub[18];
        int sk = rlp_items(d, n, it[1], sub, 18);
        if (sk < 0) return NS_BAD_RLP;
        int64_t enc = rlp_canon_len(d, n, start, 0);
        if (!((sk == 2 || sk == 17) && enc >= 0 && enc <= 31)) return NS_BAD_CHILD;
        if (sp >= 16) return NS_BAD_RLP;
        stack[sp++] = start;
      }
    } else {
      return NS_NOT_NODE;
    }
  }
  return NS_OK;
}

KH_HD bool bytes_eq32(const uint8_t* a, const uint8_t* b) {
  for (int i = 0; i < 32; ++i)
    if (a[i] != b[i]) return false;
  return true;
}

// Account.EMPTY_CODE_HASH = kec256("") and EMPTY_STATE_ROOT_HASH = kec256(0x80)
// (Account.scala:13-17)
KH_HD const uint8_t* empty_code_hash() {
  static const uint8_t h[32] = {0xc5, 0xd2, 0x46, 0x01, 0x86, 0xf7, 0x23, 0x3c, 0x92, 0x7e, 0x7d,
                                0xb2, 0xdc, 0xc7, 0x03, 0xc0, 0xe5, 0x00, 0xb6, 0x53, 0xca, 0x82,
                                0x27, 0x3b, 0x7b, 0xfa, 0xd8, 0x04, 0x5d, 0x85, 0xa4, 0x70};
  return h;
}
KH_HD const uint8_t* empty_root_hash() {
  static const uint8_t h[32] = {0x56, 0xe8, 0x1f, 0x17, 0x1b, 0xcc, 0x55, 0xa6, 0xff, 0x83, 0x45,
                                0xe6, 0x92, 0xc0, 0xf8, 0x6e, 0x5b, 0x48, 0xe0, 0x1b, 0x99, 0x6c,
                                0xad, 0xc0, 0x01, 0x62, 0x2f, 0xb5, 0xe3, 0x63, 0xb4, 0x21};
  return h;
}

// Decode value d[0, n) of a matched request of `kind` and list its children:
// out32[16*32] child hashes, kinds[16], *nchild.  Returns a NodeStatus.
KH_HD uint8_t op_node_children(const uint8_t* d, uint32_t n, uint8_t kind, uint8_t* out32, uint8_t* kinds,
                               uint8_t* nchild) {
  *nchild = 0;
  if (kind == NK_CODE || kind == NK_NONE) return NS_OK;  // EvmcodeHash: no decode
  RItem top;
  if (!rlp_valid(d, n, 0, 0) || !rlp_at(d, n, 0, top)) return NS_BAD_RLP;
  if (!top.list) return NS_NOT_NODE;
  RItem it[18];
  int k = rlp_items(d, n, top, it, 18);
  if (k < 0) return NS_BAD_RLP;
  const uint8_t child_kind = kind == NK_STATE ? NK_STATE : NK_CONTRACT;
  uint8_t cnt = 0;
  auto add = [&](uint32_t off, uint8_t kd) {
    for (int i = 0; i < 32; ++i) out32[32 * cnt + i] = d[off + i];
    kinds[cnt++] = kd;
  };
  if (k == 17) {  // MptBranch
    for (int c = 0; c < 16; ++c) {
      if (!it[c].list) {
        if (it[c].len == 32)
          add(it[c].off, child_kind);
        else if (it[c].len != 0)
          return NS_BAD_CHILD;
      } else {
        uint32_t start = c ? it[c - 1].next : top.off;
        RItem sub[18];
        int sk = rlp_items(d, n, it[c], sub, 18);
        if (sk < 0) return NS_BAD_RLP;
        int64_t enc = rlp_canon_len(d, n, start, 0);
        if (!((sk == 2 || sk == 17) && enc >= 0 && enc <= 31)) return NS_BAD_CHILD;
        uint8_t s = check_inline_node(d, n, start);
        if (s) return s;
      }
    }
    if (it[16].list) return NS_BAD_RLP;
  } else if (k == 2) {
    if (it[0].list || it[0].len == 0) return NS_BAD_RLP;
    bool leaf = (d[it[0].off] & 0x20) != 0;
    if (leaf) {
      if (it[1].list) return NS_BAD_RLP;
      if (kind == NK_STATE) {  // getAccount: RLPList(nonce, balance, stateRoot, codeHash)
        RItem a;
        if (!rlp_at(d, it[1].off + it[1].len, it[1].off, a)) return NS_BAD_ACCOUNT;
        if (!a.list) return NS_BAD_ACCOUNT;
        RItem f[5];
        int fk = rlp_items(d, it[1].off + it[1].len, a, f, 5);
        if (fk != 4) return NS_BAD_ACCOUNT;
        for (int q = 0; q < 4; ++q)
          if (f[q].list) return NS_BAD_ACCOUNT;
        if (f[0].len > 32 || f[1].len > 32) return NS_BAD_ACCOUNT;  // DataWord
        if (f[2].len != 32 || f[3].len != 32) return NS_BAD_ACCOUNT;
        if (!bytes_eq32(d + f[3].off, empty_code_hash())) add(f[3].off, NK_CODE);
        if (!bytes_eq32(d + f[2].off, empty_root_hash())) add(f[2].off, NK_STORAGE_ROOT);
      }
    } else {  // MptExtension
      if (!it[1].list) {
        if (it[1].len == 32)
          add(it[1].off, child_kind);
        else if (it[1].len != 0)
          return NS_BAD_CHILD;
      } else {
        uint32_t start = it[0].next;
        RItem sub[18];
        int sk = rlp_items(d, n, it[1], sub, 18);
        if (sk < 0) return NS_BAD_RLP;
        int64_t enc = rlp_canon_len(d, n, start, 0);
        if (!((sk == 2 || sk == 17) && enc >= 0 && enc <= 31)) return NS_BAD_CHILD;
        uint8_t s = check_inline_node(d, n, start);
        if (s) return s;
      }
    }
  } else {
    return NS_NOT_NODE;
  }
  *nchild = cnt;
  return NS_OK;
}

}  // namespace khst
