// ORACLE — TEST INFRASTRUCTURE ONLY.
//
// CPU restatement of khipu's Merkle-Patricia-trie hot path, used ONLY as the
// parity checker by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
// leg.  Nothing in khipu_amd/ links, loads or calls this file.  The product path
// (libkhst.so, HIP) fails loudly when its extension is missing; it never falls
// back to this code.
//
// The reference (Scala 2.12 / JVM) cannot be built in this image (no JDK/sbt),
// so this is a behaviour-for-behaviour restatement of the reference files below,
// pinned by the in-tree known answers (see tests/test_oracle.py):
//   kec256("")   = c5d24601...a470   (khipu-eth/.../domain/Account.scala:16)
//   kec256(0x80) = 56e81f17...b421   (Account.scala:13, trie/package.scala:41)
//   kec256(0xc0) = 1dcc4de8...9347   (domain/BlockHeader.scala:14)
//   mainnet genesis state root d7f8974f...0580f0544 over default-genesis.json
//   (GenesisDataLoader.scala:139-147) and the genesis block hash d4e56740...8fa3
//   (network/handshake/EtcHandshake.scala:52), which pins the full 32-byte root.
//
// Paths below are relative to /root/reference/khipu-base/src/main/scala/khipu/.
#include <cstdint>
#include <cstring>
#include <string>
#include <vector>
#include <array>
#include <memory>
#include <optional>
#include <unordered_map>
#include <map>
#include <stdexcept>
#include <algorithm>

namespace orc {

using Bytes = std::string;  // raw bytes; std::string so it can key hash maps

// ---------------------------------------------------------------------------
// Keccak-256, legacy padding.  crypto/hash/KeccakCore.scala:39-52 (RC),
// :103-531 (processBlock; lane-complemented form, same permutation),
// :534-562 (doPadding: 0x81 when one byte is left, else 0x01 .. 0x80),
// :570 (block length 200 - 2*32 = 136), DigestEngine.scala:102-166 (update).
// The lane-complement transform of KeccakCore (:549-554, :578-583) is an
// implementation trick whose output equals the plain permutation; this
// restatement uses the plain permutation.  `pad` selects the domain byte so the
// permutation can be cross-checked against FIPS SHA3-256 (pad 0x06).
// ---------------------------------------------------------------------------
static const uint64_t RC[24] = {
    0x0000000000000001ULL, 0x0000000000008082ULL, 0x800000000000808AULL, 0x8000000080008000ULL,
    0x000000000000808BULL, 0x0000000080000001ULL, 0x8000000080008081ULL, 0x8000000000008009ULL,
    0x000000000000008AULL, 0x0000000000000088ULL, 0x0000000080008009ULL, 0x000000008000000AULL,
    0x000000008000808BULL, 0x800000000000008BULL, 0x8000000000008089ULL, 0x8000000000008003ULL,
    0x8000000000008002ULL, 0x8000000000000080ULL, 0x000000000000800AULL, 0x800000008000000AULL,
    0x8000000080008081ULL, 0x8000000000008080ULL, 0x0000000080000001ULL, 0x8000000080008008ULL};
static const int ROT[25] = {0, 1, 62, 28, 27, 36, 44, 6, 55, 20, 3, 10, 43,
                            25, 39, 41, 45, 15, 21, 8, 18, 2, 61, 56, 14};

static inline uint64_t rotl(uint64_t x, int n) { return n ? (x << n) | (x >> (64 - n)) : x; }

uint64_t g_perms = 0;  // permutation counter (work accounting for the CPU baseline)

static void keccakf(uint64_t A[25]) {
  ++g_perms;
  for (int r = 0; r < 24; ++r) {
    uint64_t C[5], D[5], B[25];
    for (int x = 0; x < 5; ++x) C[x] = A[x] ^ A[x + 5] ^ A[x + 10] ^ A[x + 15] ^ A[x + 20];
    for (int x = 0; x < 5; ++x) D[x] = C[(x + 4) % 5] ^ rotl(C[(x + 1) % 5], 1);
    for (int i = 0; i < 25; ++i) A[i] ^= D[i % 5];
    // rho + pi: B[y, 2x+3y] = rot(A[x, y], r[x, y])
    for (int x = 0; x < 5; ++x)
      for (int y = 0; y < 5; ++y) B[y + 5 * ((2 * x + 3 * y) % 5)] = rotl(A[x + 5 * y], ROT[x + 5 * y]);
    for (int y = 0; y < 5; ++y)
      for (int x = 0; x < 5; ++x)
        A[x + 5 * y] = B[x + 5 * y] ^ ((~B[(x + 1) % 5 + 5 * y]) & B[(x + 2) % 5 + 5 * y]);
    A[0] ^= RC[r];
  }
}

void keccak256_pad(const uint8_t* in, size_t len, uint8_t pad, uint8_t out[32]) {
  uint64_t A[25] = {0};
  const size_t R = 136;
  while (len >= R) {  // DigestEngine.update: a full block is processed as soon as it fills
    for (size_t i = 0; i < R / 8; ++i) {
      uint64_t w;
      memcpy(&w, in + 8 * i, 8);
      A[i] ^= w;
    }
    keccakf(A);
    in += R;
    len -= R;
  }
  uint8_t buf[136];
  memset(buf, 0, sizeof buf);
  memcpy(buf, in, len);
  // KeccakCore.doPadding (:537-546): ptr+1 == 136 -> single byte 0x81 (pad|0x80)
  buf[len] ^= pad;
  buf[R - 1] ^= 0x80;
  for (size_t i = 0; i < R / 8; ++i) {
    uint64_t w;
    memcpy(&w, buf + 8 * i, 8);
    A[i] ^= w;
  }
  keccakf(A);
  memcpy(out, A, 32);  // encodeLELong of lanes 0..3 (:555-561)
}

Bytes kec256(const Bytes& b) {
  uint8_t o[32];
  keccak256_pad((const uint8_t*)b.data(), b.size(), 0x01, o);
  return Bytes((const char*)o, 32);
}

// ---------------------------------------------------------------------------
// RLP.  rlp/RLP.scala:116-152 (encode), :157-169 (encodeLength),
// :179-230 (getItemBounds / decodeWithPos), :285-294 (bigEndianMinLengthToInt).
// ---------------------------------------------------------------------------
struct RLPException : std::runtime_error {
  using std::runtime_error::runtime_error;
};

static Bytes encodeLength(size_t length, int offset) {
  if (length < 56) return Bytes(1, (char)(length + offset));
  if (length > 0xFF) {
    Bytes be;
    for (size_t v = length; v; v >>= 8) be.insert(be.begin(), (char)(v & 0xFF));
    return Bytes(1, (char)(be.size() + offset + 55)) + be;
  }
  Bytes r(2, 0);
  r[0] = (char)(1 + offset + 55);
  r[1] = (char)length;
  return r;
}
Bytes rlpStr(const Bytes& b) {  // RLP.scala:141-150
  if (b.size() == 1 && (uint8_t)b[0] < 0x80) return b;
  return encodeLength(b.size(), 0x80) + b;
}
Bytes rlpList(const Bytes& payload) { return encodeLength(payload.size(), 0xc0) + payload; }

struct Item {
  bool isList = false;
  Bytes bytes;
  std::vector<Item> items;
};

static uint32_t beInt(const uint8_t* p, size_t n) {
  if (n > 4) throw RLPException("Bytes don't represent an int");
  uint32_t v = 0;
  for (size_t i = 0; i < n; ++i) v = (v << 8) | p[i];
  return v;
}

static Item decodeAt(const Bytes& d, size_t pos, size_t* next);
static Item decodeAt(const Bytes& d, size_t pos, size_t* next) {
  if (d.empty()) throw RLPException("Empty Data");
  if (pos >= d.size()) throw RLPException("out of range");
  const uint8_t* u = (const uint8_t*)d.data();
  unsigned prefix = u[pos];
  Item it;
  size_t start, end;  // inclusive end, as ItemBounds
  if (prefix == 0x80) {
    *next = pos + 1;
    return it;
  } else if (prefix < 0x80) {
    it.bytes = d.substr(pos, 1);
    *next = pos + 1;
    return it;
  } else if (prefix <= 0xb7) {
    start = pos + 1;
    end = pos + (prefix - 0x80);
    it.bytes = d.substr(start, end + 1 - start);
    *next = end + 1;
    return it;
  } else if (prefix < 0xc0) {
    size_t ll = prefix - 0xb7;
    size_t len = beInt(u + pos + 1, ll);
    start = pos + 1 + ll;
    end = start + len - 1;
    it.bytes = d.substr(start, len);
    *next = end + 1;
    return it;
  } else {
    size_t len;
    if (prefix <= 0xf7) {
      start = pos + 1;
      len = prefix - 0xc0;
    } else {
      size_t ll = prefix - 0xf7;
      len = beInt(u + pos + 1, ll);
      start = pos + 1 + ll;
    }
    it.isList = true;
    size_t p = start, remain = len;
    while (remain) {  // decodeListRecursive (:222-230)
      size_t nx;
      it.items.push_back(decodeAt(d, p, &nx));
      if (nx - p > remain) throw RLPException("list overrun");
      remain -= (nx - p);
      p = nx;
    }
    *next = start + len;
    return it;
  }
}
Item rlpDecode(const Bytes& d) {
  size_t nx;
  return decodeAt(d, 0, &nx);
}

// ---------------------------------------------------------------------------
// Hex prefix.  trie/HexPrefix.scala:11-21 (encode), :30-39 (decode),
// :47-62 (bytesToNibbles), :70-85 (nibblesToBytes).  Nibble arrays hold one
// nibble per byte, as in the reference.
// ---------------------------------------------------------------------------
Bytes hpEncode(const Bytes& nib, bool isLeaf) {
  bool odd = nib.size() % 2 == 1;
  Bytes w;
  w.push_back((char)(2 * (isLeaf ? 1 : 0) + (odd ? 1 : 0)));
  if (!odd) w.push_back(0);
  w += nib;
  Bytes out(w.size() / 2, 0);
  for (size_t i = 0; i < out.size(); ++i) out[i] = (char)(16 * (uint8_t)w[2 * i] + (uint8_t)w[2 * i + 1]);
  return out;
}
Bytes bytesToNibbles(const Bytes& b) {
  Bytes n(b.size() * 2, 0);
  for (size_t i = 0; i < b.size(); ++i) {
    n[2 * i] = (char)(((uint8_t)b[i] >> 4) & 0xF);
    n[2 * i + 1] = (char)((uint8_t)b[i] & 0xF);
  }
  return n;
}
std::pair<Bytes, bool> hpDecode(const Bytes& src) {
  Bytes n = bytesToNibbles(src);
  if (n.empty()) throw std::runtime_error("HexPrefix.decode of empty array");
  bool t = (n[0] & 2) != 0;
  bool odd = (n[0] & 1) != 0;
  size_t fl = odd ? 1 : 2;
  return {n.substr(fl), t};
}

// ---------------------------------------------------------------------------
// Nodes.  trie/Node.scala:110-115 (encoded / hash / capped),
// :21-44 (nodeEnc), :46-102 (nodeDec), :128-192 (constructors).
// BranchNode.updateChild mutates the children array it shares with the node it
// was called on (:188-192); that aliasing is kept (shared_ptr to the array).
// ---------------------------------------------------------------------------
struct Node;
using NodeP = std::shared_ptr<Node>;
struct Ref {  // Either[Array[Byte], Node]: isHash == Left(bytes)
  bool isHash = false;
  Bytes hash;
  NodeP node;
};
using Slot = std::optional<Ref>;
using ChildArr = std::shared_ptr<std::array<Slot, 16>>;
enum Kind { LEAF, EXT, BRANCH };

struct Node {
  Kind kind;
  Bytes key;    // leaf key / extension shared key (nibbles)
  Bytes value;  // leaf value
  Ref next;     // extension
  ChildArr children;
  std::optional<Bytes> term;
  std::optional<Bytes> enc_, hash_;  // lazy vals

  const Bytes& encoded();
  const Bytes& hash() {
    if (!hash_) hash_ = kec256(encoded());
    return *hash_;
  }
  Bytes capped() { return encoded().size() < 32 ? encoded() : hash(); }
};

static NodeP mkLeaf(const Bytes& k, const Bytes& v) {
  auto n = std::make_shared<Node>();
  n->kind = LEAF;
  n->key = k;
  n->value = v;
  return n;
}
static NodeP mkExtRaw(const Bytes& k, const Ref& next) {
  auto n = std::make_shared<Node>();
  n->kind = EXT;
  n->key = k;
  n->next = next;
  return n;
}
static Ref refOf(const NodeP& child) {  // capped.length == 32 ? Left(hash) : Right(node)
  Bytes c = child->capped();
  Ref r;
  if (c.size() == 32) {
    r.isHash = true;
    r.hash = c;
  } else {
    r.node = child;
  }
  return r;
}
static NodeP mkExt(const Bytes& k, const NodeP& next) { return mkExtRaw(k, refOf(next)); }  // :128-131
static NodeP mkBranch(ChildArr ch, std::optional<Bytes> term) {
  auto n = std::make_shared<Node>();
  n->kind = BRANCH;
  n->children = ch;
  n->term = term;
  return n;
}
static ChildArr emptyChildren() { return std::make_shared<std::array<Slot, 16>>(); }
static NodeP branchWithValueOnly(const Bytes& v) { return mkBranch(emptyChildren(), v); }  // :144-146
static NodeP branchWithSingleChild(int pos, const NodeP& child, std::optional<Bytes> term) {
  auto ch = emptyChildren();
  (*ch)[pos] = refOf(child);
  return mkBranch(ch, term);
}
static NodeP branchWithSingleChildRef(int pos, const Ref& child, std::optional<Bytes> term) {
  auto ch = emptyChildren();
  (*ch)[pos] = child;
  return mkBranch(ch, term);
}
static NodeP updateChild(const NodeP& b, int pos, const NodeP& child) {  // :188-192 (aliasing kept)
  (*b->children)[pos] = refOf(child);
  return mkBranch(b->children, b->term);
}

const Bytes& Node::encoded() {
  if (enc_) return *enc_;
  Bytes payload;
  switch (kind) {
    case LEAF:
      payload = rlpStr(hpEncode(key, true)) + rlpStr(value);
      break;
    case EXT:
      payload = rlpStr(hpEncode(key, false)) + (next.isHash ? rlpStr(next.hash) : next.node->encoded());
      break;
    case BRANCH:
      for (int i = 0; i < 16; ++i) {
        const Slot& s = (*children)[i];
        if (!s)
          payload += rlpStr(Bytes());
        else if (s->isHash)
          payload += rlpStr(s->hash);
        else
          payload += s->node->encoded();
      }
      payload += rlpStr(term ? *term : Bytes());
      break;
  }
  enc_ = rlpList(payload);
  return *enc_;
}

static NodeP decodeNode(const Item& it) {  // Node.nodeDec (:46-102)
  if (!it.isList) throw std::runtime_error("Invalid Node");
  if (it.items.size() == 17) {
    auto ch = emptyChildren();
    for (int i = 0; i < 16; ++i) {
      const Item& c = it.items[i];
      if (c.isList) {
        Ref r;
        r.node = decodeNode(c);
        (*ch)[i] = r;
      } else if (!c.bytes.empty()) {
        Ref r;
        r.isHash = true;
        r.hash = c.bytes;
        (*ch)[i] = r;
      }
    }
    const Item& last = it.items[16];
    if (last.isList) throw RLPException("src is not an RLPValue");
    std::optional<Bytes> term;
    if (!last.bytes.empty()) term = last.bytes;
    return mkBranch(ch, term);
  } else if (it.items.size() == 2) {
    if (it.items[0].isList) throw RLPException("src is not an RLPValue");
    auto kp = hpDecode(it.items[0].bytes);
    if (kp.second) {
      if (it.items[1].isList) throw RLPException("src is not an RLPValue");
      return mkLeaf(kp.first, it.items[1].bytes);
    }
    Ref r;
    if (it.items[1].isList) {
      r.node = decodeNode(it.items[1]);
    } else {
      r.isHash = true;
      r.hash = it.items[1].bytes;
    }
    return mkExtRaw(kp.first, r);
  }
  throw std::runtime_error("Invalid Node");
}

// ---------------------------------------------------------------------------
// Node store: EphemNodeDataSource behind ArchiveNodeStorage
// (khipu-eth/.../storage/ArchiveNodeStorage.scala:18-20: removes are ignored).
// ---------------------------------------------------------------------------
struct Storage {
  std::unordered_map<Bytes, Bytes> m;
};

struct MPTException : std::runtime_error {
  using std::runtime_error::runtime_error;
};
struct MPTNodeMissing : std::runtime_error {
  Bytes hash;
  MPTNodeMissing(const std::string& s, const Bytes& h) : std::runtime_error(s), hash(h) {}
};

enum LogKind { ORIGINAL, UPDATED, REMOVED };
struct Log {
  LogKind k;
  Bytes v;
};
struct Change {
  bool updated;
  NodeP node;
};
using Changes = std::vector<Change>;

extern const Bytes EMPTY_TRIE_HASH;
const Bytes EMPTY_TRIE_HASH = kec256(rlpStr(Bytes()));  // trie/package.scala:41

static size_t matchingLength(const Bytes& a, const Bytes& b) {  // MerklePatriciaTrie.scala:49-55
  size_t i = 0;
  while (i < a.size() && i < b.size() && a[i] == b[i]) ++i;
  return i;
}

// MerklePatriciaTrie.scala:68-558.  A put/remove mutates this instance in place
// (the reference returns a new instance holding updateNodesToLogs(...); the
// drivers below never reuse the old one, and getNode's `nodeLogs +=` already
// mutates the shared var before the new instance is made).
struct MPT {
  std::optional<Bytes> rootHashOpt;
  Storage* storage;
  std::unordered_map<Bytes, Log> nodeLogs;

  MPT(Storage* s, const Bytes& rootHash) : storage(s) {  // :60-66
    if (rootHash != EMPTY_TRIE_HASH) rootHashOpt = rootHash;
  }
  Bytes rootHash() const { return rootHashOpt ? *rootHashOpt : EMPTY_TRIE_HASH; }  // :78

  NodeP getNode(const Bytes& id) {  // :520-542
    Bytes enc;
    if (id.size() < 32) {
      enc = id;
    } else {
      auto it = nodeLogs.find(id);
      if (it == nodeLogs.end()) {
        auto s = storage->m.find(id);
        if (s == storage->m.end()) throw MPTNodeMissing("Node not found, trie is inconsistent", id);
        nodeLogs[id] = Log{ORIGINAL, s->second};
        enc = s->second;
      } else if (it->second.k == REMOVED) {
        throw MPTNodeMissing("Node has been deleted, trie is inconsistent", id);
      } else {
        enc = it->second.v;
      }
    }
    return decodeNode(rlpDecode(enc));
  }
  NodeP nextNode(const NodeP& ext) { return ext->next.isHash ? getNode(ext->next.hash) : ext->next.node; }
  std::optional<NodeP> getChild(const NodeP& b, int pos) {
    const Slot& s = (*b->children)[pos];
    if (!s) return std::nullopt;
    return s->isHash ? getNode(s->hash) : s->node;
  }

  // --- get (:90-133)
  std::optional<Bytes> get(const Bytes& key) {
    if (!rootHashOpt) return std::nullopt;
    NodeP node = getNode(*rootHashOpt);
    Bytes sk = bytesToNibbles(key);
    for (;;) {
      if (node->kind == LEAF) {
        if (node->key == sk) return node->value;
        return std::nullopt;
      } else if (node->kind == EXT) {
        if (sk.size() >= node->key.size() && sk.compare(0, node->key.size(), node->key) == 0) {
          NodeP nx = nextNode(node);
          sk = sk.substr(node->key.size());
          node = nx;
        } else {
          return std::nullopt;
        }
      } else {
        if (sk.empty()) return node->term;
        auto c = getChild(node, sk[0]);
        if (!c) return std::nullopt;
        node = *c;
        sk = sk.substr(1);
      }
    }
  }

  // --- put (:157-281)
  struct Ins {
    NodeP n;
    Changes ch;
  };
  void put(const Bytes& key, const Bytes& value) {
    Bytes kn = bytesToNibbles(key);
    Ins r;
    if (rootHashOpt) {
      NodeP root = getNode(*rootHashOpt);
      r = put(root, kn, value);
    } else {
      NodeP nr = mkLeaf(kn, value);
      r = Ins{nr, {{true, nr}}};
    }
    Bytes prev = rootHash();
    Bytes h = r.n->hash();  // :169, the new root is always hashed (evaluated first)
    updateNodesToLogs(prev, r.n, r.ch);
    rootHashOpt = h;
  }
  Ins put(const NodeP& n, const Bytes& sk, const Bytes& v) {
    switch (n->kind) {
      case LEAF: return putInLeaf(n, sk, v);
      case EXT: return putInExt(n, sk, v);
      default: return putInBranch(n, sk, v);
    }
  }
  Ins putInLeaf(const NodeP& node, const Bytes& sk, const Bytes& v) {  // :183-219
    const Bytes& ek = node->key;
    size_t ml = matchingLength(ek, sk);
    if (ml == 0) {
      NodeP tb;
      NodeP maybeLeaf;
      if (ek.empty()) {
        tb = branchWithValueOnly(node->value);
      } else {
        maybeLeaf = mkLeaf(ek.substr(1), node->value);
        tb = branchWithSingleChild(ek[0], maybeLeaf, std::nullopt);
      }
      Ins r = put(tb, sk, v);
      r.ch.push_back({false, node});
      if (maybeLeaf) r.ch.push_back({true, maybeLeaf});
      return r;
    } else if (ml == ek.size() && ml == sk.size()) {
      NodeP nl = mkLeaf(ek, v);
      return Ins{nl, {{false, node}, {true, nl}}};
    } else {
      Bytes pre = sk.substr(0, ml), suf = sk.substr(ml);
      NodeP tmp = (ml == ek.size()) ? branchWithValueOnly(node->value) : mkLeaf(ek.substr(ml), node->value);
      Ins r = put(tmp, suf, v);
      NodeP ne = mkExt(pre, r.n);
      r.ch.push_back({false, node});
      r.ch.push_back({true, ne});
      r.n = ne;
      return r;
    }
  }
  Ins putInExt(const NodeP& ext, const Bytes& sk, const Bytes& v) {  // :221-254
    const Bytes& shk = ext->key;
    size_t ml = matchingLength(shk, sk);
    if (ml == 0) {
      int head = shk[0];
      NodeP tb, maybeExt;
      if (shk.size() == 1) {
        tb = branchWithSingleChildRef(head, ext->next, std::nullopt);
      } else {
        maybeExt = mkExtRaw(shk.substr(1), ext->next);
        tb = branchWithSingleChild(head, maybeExt, std::nullopt);
      }
      Ins r = put(tb, sk, v);
      r.ch.push_back({false, ext});
      if (maybeExt) r.ch.push_back({true, maybeExt});
      return r;
    } else if (ml == shk.size()) {
      Ins r = put(nextNode(ext), sk.substr(ml), v);
      NodeP ne = mkExt(shk, r.n);
      r.ch.push_back({false, ext});
      r.ch.push_back({true, ne});
      r.n = ne;
      return r;
    } else {
      Bytes pre = shk.substr(0, ml), suf = shk.substr(ml);
      NodeP tmpExt = mkExtRaw(suf, ext->next);
      Ins r = put(tmpExt, sk.substr(ml), v);
      NodeP ne = mkExt(pre, r.n);
      r.ch.push_back({false, ext});
      r.ch.push_back({true, ne});
      r.n = ne;
      return r;
    }
  }
  Ins putInBranch(const NodeP& b, const Bytes& sk, const Bytes& v) {  // :256-281
    if (sk.empty()) {
      NodeP nb = mkBranch(b->children, v);
      return Ins{nb, {{false, b}, {true, nb}}};
    }
    int head = sk[0];
    Bytes tail = sk.substr(1);
    if ((*b->children)[head]) {
      NodeP child = *getChild(b, head);
      Ins r = put(child, tail, v);
      NodeP nb = updateChild(b, head, r.n);
      r.ch.push_back({false, b});
      r.ch.push_back({true, nb});
      r.n = nb;
      return r;
    }
    NodeP nl = mkLeaf(tail, v);
    NodeP nb = updateChild(b, head, nl);
    return Ins{nb, {{false, b}, {true, nl}, {true, nb}}};
  }

  // --- remove (:290-416)
  struct Rem {
    bool changed;
    NodeP n;  // null == None
    Changes ch;
  };
  void remove(const Bytes& key) {
    if (!rootHashOpt) return;
    Bytes kn = bytesToNibbles(key);
    NodeP root = getNode(*rootHashOpt);
    Rem r = remove(root, kn);
    if (!r.changed) return;
    Bytes prev = rootHash();
    std::optional<Bytes> h;
    if (r.n) h = r.n->hash();  // :298
    updateNodesToLogs(prev, r.n, r.ch);
    rootHashOpt = h;
  }
  Rem remove(const NodeP& n, const Bytes& sk) {
    switch (n->kind) {
      case LEAF:
        if (n->key == sk) return Rem{true, nullptr, {{false, n}}};
        return Rem{false, nullptr, {}};
      case EXT: return removeFromExt(n, sk);
      default: return removeFromBranch(n, sk);
    }
  }
  Rem removeFromBranch(const NodeP& node, const Bytes& sk) {  // :323-370
    if (sk.empty()) {
      if (!node->term) return Rem{false, nullptr, {}};
      NodeP fixed = fix(mkBranch(node->children, std::nullopt), {});
      return Rem{true, fixed, {{false, node}, {true, fixed}}};
    }
    int head = sk[0];
    auto child = getChild(node, head);
    if (!child) return Rem{false, nullptr, {}};
    Rem r = remove(*child, sk.substr(1));
    if (!r.changed) return Rem{false, nullptr, r.ch};
    NodeP toFix;
    if (r.n) {
      toFix = updateChild(node, head, r.n);
    } else {
      (*node->children)[head].reset();
      toFix = mkBranch(node->children, node->term);
    }
    std::vector<NodeP> upd;
    for (auto& c : r.ch)
      if (c.updated) upd.push_back(c.node);
    NodeP fixed = fix(toFix, upd);
    r.ch.push_back({false, node});
    r.ch.push_back({true, fixed});
    return Rem{true, fixed, r.ch};
  }
  Rem removeFromExt(const NodeP& ext, const Bytes& sk) {  // :383-416
    size_t ml = matchingLength(ext->key, sk);
    if (ml != ext->key.size()) return Rem{false, ext, {}};
    Rem r = remove(nextNode(ext), sk.substr(ml));
    if (!r.changed) return Rem{false, nullptr, r.ch};
    if (!r.n) throw MPTException("A trie with newRoot extension should have at least 2 values stored");
    NodeP toFix = mkExt(ext->key, r.n);
    std::vector<NodeP> upd;
    for (auto& c : r.ch)
      if (c.updated) upd.push_back(c.node);
    NodeP fixed = fix(toFix, upd);
    r.ch.push_back({false, ext});
    r.ch.push_back({true, fixed});
    return Rem{true, fixed, r.ch};
  }
  NodeP fix(NodeP node, const std::vector<NodeP>& notStoredYet) {  // :430-477
    for (;;) {
      if (node->kind == BRANCH) {
        std::vector<int> used;
        for (int i = 0; i < 16; ++i)
          if ((*node->children)[i]) used.push_back(i);
        if (used.empty() && !node->term) throw MPTException("Branch with no subvalues");
        if (used.size() == 1 && !node->term) {
          int idx = used[0];
          node = mkExtRaw(Bytes(1, (char)idx), *(*node->children)[idx]);
          continue;  // tail call fix(temporalExtNode)
        }
        if (used.empty() && node->term) return mkLeaf(Bytes(), *node->term);
        return node;
      } else if (node->kind == EXT) {
        NodeP nx;
        if (node->next.isHash) {
          for (auto& n : notStoredYet)
            if (n->hash() == node->next.hash) {
              nx = n;
              break;
            }
          if (!nx) nx = nextNode(node);
        } else {
          nx = node->next.node;
        }
        if (nx->kind == EXT) return mkExtRaw(node->key + nx->key, nx->next);
        if (nx->kind == LEAF) return mkLeaf(node->key + nx->key, nx->value);
        return node;
      }
      return node;
    }
  }

  // --- updateNodesToLogs (:491-516)
  void updateNodesToLogs(const Bytes& prevRootHash, const NodeP& newRoot, const Changes& changes) {
    std::unordered_map<Bytes, Change> dedup;
    for (auto& c : changes) dedup[c.node->hash()] = c;  // later entries win
    Bytes rootCapped = newRoot ? newRoot->capped() : Bytes();
    std::vector<std::pair<Bytes, Log>> toRemove, toUpdate;
    for (auto& kv : dedup) {
      Bytes capped = kv.second.node->capped();
      if (!kv.second.updated) {
        if (capped.size() == 32 || kv.first == prevRootHash) toRemove.push_back({kv.first, Log{REMOVED, Bytes()}});
      } else {
        if (capped.size() == 32 || capped == rootCapped)
          toUpdate.push_back({kv.first, Log{UPDATED, kv.second.node->encoded()}});
      }
    }
    for (auto& e : toRemove) nodeLogs[e.first] = e.second;
    for (auto& e : toUpdate) nodeLogs[e.first] = e.second;
  }

  void persist() {  // :544-547 -> ArchiveNodeStorage.update (removes ignored)
    for (auto& kv : nodeLogs)
      if (kv.second.k == UPDATED) storage->m[kv.first] = kv.second.v;
  }
};

}  // namespace orc

// ---------------------------------------------------------------------------
// C ABI for ctypes (tests / bench cpu_baseline only).
// ---------------------------------------------------------------------------
using namespace orc;

struct or_trie {
  Storage own;
  Storage* st;
  MPT mpt;
  std::string err;
  or_trie() : st(&own), mpt(&own, EMPTY_TRIE_HASH) {}
};

// ---------------------------------------------------------------------------
// Fast-sync NodeData decode: PV63.MptNode decoding
// (network/p2p/messages/PV63.scala:96-127) and the child-hash lists of
// NodeDatasRequest (blockchain/sync/package.scala:127-165).  RLP items are decoded
// strictly: a truncated item is an error here (the reference's copyOfRange would
// zero-pad it), reported with the status codes of include/khst.h kh_verify_nodes.
// ---------------------------------------------------------------------------
struct NodeErr {
  int status;
};
struct SItem {  // strictly decoded RLP item
  bool isList = false;
  Bytes bytes;
  std::vector<SItem> items;
};
static SItem sdecode(const Bytes& d, size_t pos, size_t end, size_t* next) {
  if (pos >= end) throw NodeErr{4};
  const uint8_t* u = (const uint8_t*)d.data();
  unsigned p = u[pos];
  size_t off, len;
  bool list;
  if (p < 0x80) {
    off = pos, len = 1, list = false;
  } else if (p <= 0xb7) {
    off = pos + 1, len = p - 0x80, list = false;
  } else if (p <= 0xbf || p >= 0xf8) {
    size_t ll = p <= 0xbf ? p - 0xb7 : p - 0xf7;
    if (ll > 4 || pos + 1 + ll > end) throw NodeErr{4};
    len = 0;
    for (size_t i = 0; i < ll; ++i) len = (len << 8) | u[pos + 1 + i];
    off = pos + 1 + ll, list = p >= 0xc0;
  } else {
    off = pos + 1, len = p - 0xc0, list = true;
  }
  if (off + len > end) throw NodeErr{4};
  SItem it;
  it.isList = list;
  if (!list) {
    it.bytes = d.substr(off, len);
  } else {
    size_t q = off;
    while (q < off + len) {
      size_t nx;
      it.items.push_back(sdecode(d, q, off + len, &nx));
      q = nx;
    }
  }
  *next = off + len;
  return it;
}
static Bytes sencode(const SItem& it) {  // rlp.encode (canonical)
  if (!it.isList) return rlpStr(it.bytes);
  Bytes pl;
  for (auto& c : it.items) pl += sencode(c);
  return rlpList(pl);
}
static void mptNodeCheck(const SItem& it);
// decodeChild (PV63.scala:113-125): true = Left(MptHash), false = Right(node)
static bool decodeChild(const SItem& c) {
  if (!c.isList && (c.bytes.size() == 32 || c.bytes.empty())) return true;
  size_t enc = sencode(c).size();
  if (c.isList && (c.items.size() == 2 || c.items.size() == 17) && enc <= 31) {
    mptNodeCheck(c);
    return false;
  }
  throw NodeErr{2};
}
// toMptNode (PV63.scala:99-111), for its exceptions only
static void mptNodeCheck(const SItem& it) {
  if (it.isList && it.items.size() == 17) {
    for (int i = 0; i < 16; ++i) decodeChild(it.items[i]);
    if (it.items[16].isList) throw NodeErr{4};
    return;
  }
  if (it.isList && it.items.size() == 2) {
    if (it.items[0].isList || it.items[0].bytes.empty()) throw NodeErr{4};
    bool leaf = (((uint8_t)it.items[0].bytes[0] >> 4) & 2) != 0;
    if (leaf) {
      if (it.items[1].isList) throw NodeErr{4};
    } else {
      decodeChild(it.items[1]);
    }
    return;
  }
  throw NodeErr{1};
}
// kind: 0 state node, 1 storage root, 2 contract storage node, 3 evm code
static int nodeChildren(const Bytes& v, int kind, std::vector<std::pair<Bytes, int>>& out) {
  if (kind == 3) return 0;
  try {
    size_t nx;
    SItem it = sdecode(v, 0, v.size(), &nx);
    const int ck = kind == 0 ? 0 : 2;  // StateMptNodeHash / ContractStorageMptNodeHash
    if (it.isList && it.items.size() == 17) {  // MptBranch: Left hashes, nonEmpty
      std::vector<std::pair<Bytes, int>> kids;
      for (int i = 0; i < 16; ++i)
        if (decodeChild(it.items[i]) && !it.items[i].bytes.empty()) kids.push_back({it.items[i].bytes, ck});
      if (it.items[16].isList) throw NodeErr{4};
      out = kids;
      return 0;
    }
    if (it.isList && it.items.size() == 2) {
      if (it.items[0].isList || it.items[0].bytes.empty()) throw NodeErr{4};
      bool leaf = (((uint8_t)it.items[0].bytes[0] >> 4) & 2) != 0;
      if (leaf) {
        if (it.items[1].isList) throw NodeErr{4};
        if (kind != 0) return 0;  // getContractMptNodeChildren: a leaf has none
        // getAccount: rawDecode(value) = RLPList(nonce, balance, stateRoot, codeHash)
        const Bytes& val = it.items[1].bytes;
        SItem a;
        try {
          size_t n2;
          a = sdecode(val, 0, val.size(), &n2);
        } catch (NodeErr&) {
          throw NodeErr{3};
        }
        if (!a.isList || a.items.size() != 4) throw NodeErr{3};
        for (auto& f : a.items)
          if (f.isList) throw NodeErr{3};
        if (a.items[0].bytes.size() > 32 || a.items[1].bytes.size() > 32) throw NodeErr{3};  // DataWord
        if (a.items[2].bytes.size() != 32 || a.items[3].bytes.size() != 32) throw NodeErr{3};
        static const Bytes EMPTY_CODE = kec256(Bytes());
        if (a.items[3].bytes != EMPTY_CODE) out.push_back({a.items[3].bytes, 3});       // EvmcodeHash
        if (a.items[2].bytes != EMPTY_TRIE_HASH) out.push_back({a.items[2].bytes, 1});  // StorageRootHash
        return 0;
      }
      // MptExtension: Left(hash) -> the hash; Right(node) -> none
      if (decodeChild(it.items[1]) && !it.items[1].bytes.empty()) out.push_back({it.items[1].bytes, ck});
      return 0;
    }
    if (!it.isList) throw NodeErr{1};
    throw NodeErr{1};
  } catch (NodeErr& e) {
    out.clear();
    return e.status;
  }
}

static thread_local std::string g_err;

extern "C" {

const char* or_last_error() { return g_err.c_str(); }
uint64_t or_perm_count() { return g_perms; }
void or_perm_reset() { g_perms = 0; }

void or_keccak256_pad(const uint8_t* in, uint64_t len, uint8_t pad, uint8_t* out32) {
  keccak256_pad(in, (size_t)len, pad, out32);
}
void or_kec256(const uint8_t* in, uint64_t len, uint8_t* out32) { keccak256_pad(in, (size_t)len, 0x01, out32); }

// RLP helpers exposed for unit tests of the encoding contract.
int64_t or_rlp_str(const uint8_t* in, uint64_t len, uint8_t* out, uint64_t cap) {
  Bytes r = rlpStr(Bytes((const char*)in, len));
  if (r.size() > cap) return -(int64_t)r.size();
  memcpy(out, r.data(), r.size());
  return (int64_t)r.size();
}
int64_t or_rlp_list(const uint8_t* payload, uint64_t len, uint8_t* out, uint64_t cap) {
  Bytes r = rlpList(Bytes((const char*)payload, len));
  if (r.size() > cap) return -(int64_t)r.size();
  memcpy(out, r.data(), r.size());
  return (int64_t)r.size();
}
int64_t or_hp_encode(const uint8_t* nibbles, uint64_t n, int is_leaf, uint8_t* out, uint64_t cap) {
  Bytes r = hpEncode(Bytes((const char*)nibbles, n), is_leaf != 0);
  if (r.size() > cap) return -(int64_t)r.size();
  memcpy(out, r.data(), r.size());
  return (int64_t)r.size();
}

or_trie* or_trie_new() { return new or_trie(); }
void or_trie_free(or_trie* t) { delete t; }

#define OR_TRY(body)                 \
  try {                              \
    body;                            \
    return 0;                        \
  } catch (MPTNodeMissing & e) {     \
    g_err = e.what();                \
    return -3;                       \
  } catch (std::exception & e) {     \
    g_err = e.what();                \
    return -1;                       \
  }

int or_trie_put(or_trie* t, const uint8_t* k, uint64_t kl, const uint8_t* v, uint64_t vl) {
  OR_TRY(t->mpt.put(Bytes((const char*)k, kl), Bytes((const char*)v, vl)))
}
int or_trie_remove(or_trie* t, const uint8_t* k, uint64_t kl) { OR_TRY(t->mpt.remove(Bytes((const char*)k, kl))) }
// returns value length, -2 if absent, <0 on error; copies min(len, cap) bytes
int64_t or_trie_get(or_trie* t, const uint8_t* k, uint64_t kl, uint8_t* out, uint64_t cap) {
  try {
    auto r = t->mpt.get(Bytes((const char*)k, kl));
    if (!r) return -2;
    memcpy(out, r->data(), std::min<uint64_t>(cap, r->size()));
    return (int64_t)r->size();
  } catch (std::exception& e) {
    g_err = e.what();
    return -1;
  }
}
void or_trie_root(or_trie* t, uint8_t* out32) {
  Bytes r = t->mpt.rootHash();
  memcpy(out32, r.data(), 32);
}
void or_trie_persist(or_trie* t) { t->mpt.persist(); }
// Re-open the trie at its current root against the same store with empty logs
// (what GenesisDataLoader does per account: new MPT(rootHash, storage)).
void or_trie_reopen(or_trie* t) {
  Bytes r = t->mpt.rootHash();
  t->mpt = MPT(t->st, r);
}
// Number of Updated log entries (the write-back set, MerklePatriciaTrie.changes :549-554)
uint64_t or_trie_updated_count(or_trie* t) {
  uint64_t c = 0;
  for (auto& kv : t->mpt.nodeLogs)
    if (kv.second.k == UPDATED) ++c;
  return c;
}
// Dump Updated entries: hashes (32 B each) + concatenated encodings with offsets[n+1].
int or_trie_updated_dump(or_trie* t, uint8_t* hashes, uint8_t* enc, uint64_t enc_cap, uint64_t* off) {
  std::map<Bytes, Bytes> sorted;
  for (auto& kv : t->mpt.nodeLogs)
    if (kv.second.k == UPDATED) sorted[kv.first] = kv.second.v;
  uint64_t i = 0, o = 0;
  off[0] = 0;
  for (auto& kv : sorted) {
    memcpy(hashes + 32 * i, kv.first.data(), 32);
    if (o + kv.second.size() > enc_cap) return -1;
    memcpy(enc + o, kv.second.data(), kv.second.size());
    o += kv.second.size();
    off[++i] = o;
  }
  return 0;
}
uint64_t or_trie_store_size(or_trie* t) { return t->st->m.size(); }

// Nodes reachable from the current root whose encoding is >= 32 B, plus the root
// (i.e. every node a fresh store needs).  Sorted by hash.
int64_t or_trie_reachable(or_trie* t, uint8_t* hashes, uint64_t hcap, uint8_t* enc, uint64_t enc_cap, uint64_t* off) {
  try {
    std::map<Bytes, Bytes> out;
    if (t->mpt.rootHashOpt) {
      std::vector<std::pair<Bytes, NodeP>> stack;
      NodeP root = t->mpt.getNode(*t->mpt.rootHashOpt);
      out[root->hash()] = root->encoded();
      stack.push_back({Bytes(), root});
      while (!stack.empty()) {
        NodeP n = stack.back().second;
        stack.pop_back();
        auto visit = [&](const Ref& r) {
          NodeP c = r.isHash ? t->mpt.getNode(r.hash) : r.node;
          if (c->encoded().size() >= 32) out[c->hash()] = c->encoded();
          stack.push_back({Bytes(), c});
        };
        if (n->kind == EXT) visit(n->next);
        if (n->kind == BRANCH)
          for (auto& s : *n->children)
            if (s) visit(*s);
      }
    }
    if (!hashes) return (int64_t)out.size();
    uint64_t i = 0, o = 0;
    off[0] = 0;
    for (auto& kv : out) {
      if (i >= hcap || o + kv.second.size() > enc_cap) return -1;
      memcpy(hashes + 32 * i, kv.first.data(), 32);
      memcpy(enc + o, kv.second.data(), kv.second.size());
      o += kv.second.size();
      off[++i] = o;
    }
    return (int64_t)i;
  } catch (std::exception& e) {
    g_err = e.what();
    return -1;
  }
}

// Sequential batch: the TrieAccounts.flush pattern (TrieAccounts.scala:22-28):
// one trie instance, foldLeft of put (or remove when `is_del[i]`), then rootHash.
// keys: n * klen bytes; vals packed with voff[n+1].  mode bit 1 = GenesisDataLoader
// pattern (GenesisDataLoader.scala:139-147): a fresh instance per put, persist
// after each; mode bit 2 = the key is kec256 of the given bytes, hashed inside the
// loop (Address.hashedAddressEncoder, Address.scala:15-17).
int or_seq_root(const uint8_t* keys, uint64_t klen, const uint8_t* vals, const uint64_t* voff, const uint8_t* is_del,
                uint64_t n, int mode, uint8_t* out32) {
  try {
    Storage st;
    MPT m(&st, EMPTY_TRIE_HASH);
    const bool genesis = (mode & 1) != 0;
    const bool hash_keys = (mode & 2) != 0;  // key = kec256(key bytes): Address.hashedAddressEncoder
    for (uint64_t i = 0; i < n; ++i) {
      if (genesis) m = MPT(&st, m.rootHash());
      Bytes k((const char*)keys + i * klen, klen);
      if (hash_keys) {
        uint8_t h[32];
        keccak256_pad((const uint8_t*)k.data(), k.size(), 0x01, h);
        k.assign((const char*)h, 32);
      }
      if (is_del && is_del[i])
        m.remove(k);
      else
        m.put(k, Bytes((const char*)vals + voff[i], voff[i + 1] - voff[i]));
      if (genesis) m.persist();
    }
    Bytes r = m.rootHash();
    memcpy(out32, r.data(), 32);
    return 0;
  } catch (std::exception& e) {
    g_err = e.what();
    return -1;
  }
}

// fast-sync decode of one value: status (kh_verify_nodes codes); children into
// out32 (16 x 32 B) and kinds, count into *n
int or_node_children(const uint8_t* v, uint64_t len, int kind, uint8_t* out32, uint8_t* kinds, uint32_t* n) {
  std::vector<std::pair<Bytes, int>> ch;
  int st = nodeChildren(Bytes((const char*)v, len), kind, ch);
  *n = (uint32_t)ch.size();
  for (size_t i = 0; i < ch.size() && i < 16; ++i) {
    memcpy(out32 + 32 * i, ch[i].first.data(), 32);
    kinds[i] = (uint8_t)ch[i].second;
  }
  return st;
}

// NodeDatasRequest.processResponse (sync/package.scala:81-125) over one batch, one core: kec256
// of every value, the request it answers (requestNodeHashes.map(...).toMap: the last request of
// equal hashes wins), and for a matched trie node its PV63 decode and child list
// (getStateNodeChildren / getContractMptNodeChildren, :127-165).  Outputs laid out as
// kh_verify_nodes' (include/khst.h): the CPU leg of bench.py --workload verify.
int or_verify_nodes(const uint8_t* data, const uint64_t* off, uint64_t n, const uint8_t* req32, const uint8_t* req_kind,
                    uint64_t nreq, uint8_t* hash32, int64_t* match, uint8_t* status, uint8_t* nchild, uint8_t* child32,
                    uint8_t* child_kind) {
  std::unordered_map<std::string, int64_t> req;
  req.reserve(nreq * 2 + 1);
  for (uint64_t r = 0; r < nreq; ++r) req[std::string((const char*)req32 + 32 * r, 32)] = (int64_t)r;
  for (uint64_t i = 0; i < n; ++i) {
    const uint8_t* v = data + off[i];
    const uint64_t len = off[i + 1] - off[i];
    uint8_t h[32];
    keccak256_pad(v, (size_t)len, 0x01, h);
    memcpy(hash32 + 32 * i, h, 32);
    auto it = req.find(std::string((const char*)h, 32));
    match[i] = it == req.end() ? -1 : it->second;
    status[i] = 0;
    nchild[i] = 0;
    if (it == req.end()) continue;
    const int kind = req_kind[it->second];
    if (kind == 3) continue;  // EvmcodeHash: no decoding
    uint32_t nc = 0;
    status[i] = (uint8_t)or_node_children(v, len, kind, child32 + 512 * i, child_kind + 16 * i, &nc);
    nchild[i] = (uint8_t)nc;
  }
  return 0;
}

}  // extern "C"
