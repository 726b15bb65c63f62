// libkhst.so — MI355X batch state-root engine for khipu's Merkle-Patricia trie.
// HIP kernels for gfx950 + the C ABI declared in include/khst.h.
//
// Pipeline of one build (all on one HIP stream; DESIGN.md has the roofline of each):
//   1. keys      kec256 of raw keys (KH_HASH_KEYS)                       k_hash_keys
//   2. sort      32-bit prefix LSD radix sort of (segment|key prefix, index) prims.h
//                + local full-key sort of equal-prefix runs, dedup        k_tie_fix/k_dup
//                (full 256-bit sort only for runs > 64: adversarial keys)
//   3. topology  adjacent LCP -> min pyramid -> nearest smaller values
//                -> groups (branches), parents, child ordinals            k_lcp..k_leaf_topo
//   4. leaves    RLP-encode into the node arena, then Keccak-256          k_leaf_prep/hash
//   5. branches  per depth, deepest first: gather child refs and RLP-encode,
//                then Keccak-256 (+ extension)                            k_branch_prep/hash
// Results: the top node of every segment (root / subtrie reference).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <condition_variable>
#include <exception>
#include <functional>
#include <memory>
#include <mutex>
#include <thread>
#include <string>
#include <vector>

#include "../../include/khst.h"
#include "keccak.h"
#include "keccak_xlane.h"
#include "prims.h"
#include "synth.h"
#include "trie_ops.h"
#include "keyorder.h"
#include "forest.h"
#include "nodedata.h"

using namespace khst;

// ---------------------------------------------------------------------------
// errors
// ---------------------------------------------------------------------------
static thread_local std::string g_err;
static int set_err(int code, const std::string& msg) {
  g_err = msg;
  return code;
}
struct KhError {
  int code;
  std::string msg;
};
#define HIPCHK(x)                                                                                  \
  do {                                                                                             \
    hipError_t e_ = (x);                                                                           \
    if (e_ != hipSuccess) {                                                                        \
      (void)hipGetLastError(); /* clear it, or the next launch check reports it again */           \
      throw KhError{e_ == hipErrorOutOfMemory ? KH_ENOMEM : KH_EDEVICE,                            \
                    std::string(#x) + ": " + hipGetErrorString(e_)};                               \
    }                                                                                              \
  } while (0)
#define LAUNCH_CHECK() HIPCHK(hipGetLastError())

#define GRID(n, bs) dim3((unsigned)(((n) + (bs)-1) / (bs)))
constexpr int BS = 256;

// ---------------------------------------------------------------------------
// kernels
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(BS) k_kec_batch(const uint8_t* data, const uint64_t* off, uint64_t n,
                                                  uint64_t* out) {
  uint64_t i = (uint64_t)blockIdx.x * BS + threadIdx.x;
  if (i >= n) return;
  uint64_t h[4];
  uint64_t o = off[i];
  kec256_msg<false>(data + o, (uint32_t)(off[i + 1] - o), h);
  for (int j = 0; j < 4; ++j) out[4 * i + j] = h[j];
}

// fast-sync NodeData verification (nodedata.h): hash, match against the sorted
// requested hashes (the last of equal requests wins, as Map construction does), decode
__global__ void __launch_bounds__(BS) k_verify_nodes(const uint8_t* data, const uint64_t* off, uint64_t n,
                                                     const uint64_t* req, const uint8_t* req_kind,
                                                     const uint32_t* req_idx, uint64_t nreq, uint64_t* hash_out,
                                                     int64_t* match, uint8_t* status, uint32_t* nchild,
                                                     uint8_t* child32, uint8_t* child_kind) {
  // req: the distinct requested hashes in key order, req_idx: the request each stands for (the
  // last of equal hashes: requestNodeHashes.toMap, sync/package.scala:85); req_kind by request
  uint64_t i = (uint64_t)blockIdx.x * BS + threadIdx.x;
  if (i >= n) return;
  const uint64_t o = off[i];
  const uint32_t len = (uint32_t)(off[i + 1] - o);
  uint64_t h[4];
  kec256_msg<false>(data + o, len, h);
  for (int j = 0; j < 4; ++j) hash_out[4 * i + j] = h[j];
  const uint64_t p = key_lower_bound(req, nreq, h);
  int64_t mi = -1;
  uint8_t kind = NK_NONE;
  if (p < nreq && key_cmp(req + 4 * p, h) == 0) {
    mi = req_idx[p];
    kind = req_kind[mi];
  }
  match[i] = mi;
  uint8_t nc = 0;
  status[i] = op_node_children(data + o, len, kind, child32 + 512 * i, child_kind + 16 * i, &nc);
  nchild[i] = nc;
}
__global__ void __launch_bounds__(BS) k_u32_to_u64(const uint32_t* in, uint64_t n, uint64_t* out) {
  const uint64_t i = (uint64_t)blockIdx.x * BS + threadIdx.x;
  if (i < n) out[i] = in[i];
}
__global__ void k_set_last(uint64_t* dst, const uint64_t* src) { *dst = *src; }
// the children of value i packed at coff[i] (the exclusive scan of the counts)
__global__ void __launch_bounds__(BS) k_pack_children(const uint32_t* nchild, const uint64_t* coff, uint64_t n,
                                                      const uint8_t* child32, const uint8_t* child_kind,
                                                      uint8_t* out32, uint8_t* out_kind) {
  const uint64_t g = (uint64_t)blockIdx.x * BS + threadIdx.x, i = g >> 4;
  const uint32_t c = (uint32_t)(g & 15);  // 16 threads per value: one child each
  if (i >= n || c >= nchild[i]) return;
  const uint64_t d = coff[i] + c;
  const ulonglong2* src = (const ulonglong2*)(child32 + 512 * i + 32 * c);
  ulonglong2* dst = (ulonglong2*)(out32 + 32 * d);
  dst[0] = src[0];
  dst[1] = src[1];
  out_kind[d] = child_kind[16 * i + c];
}

template <bool SHORT>
__global__ void __launch_bounds__(BS) k_hash_keys(const uint8_t* keys, uint32_t klen, uint64_t n, uint64_t* out) {
  uint64_t i = (uint64_t)blockIdx.x * BS + threadIdx.x;
  if (i >= n) return;
  uint64_t h[4];
  if (SHORT)
    kec256_short(keys + i * klen, klen, h);
  else
    kec256_msg<false>(keys + i * klen, klen, h);
  for (int j = 0; j < 4; ++j) out[4 * i + j] = h[j];
}

// ... and the unsegmented sort key (the key's leading 32 bits, big-endian) with the
// identity index in the same pass (saves k_make_ck's re-read of the keys)
#ifndef KH_KEYS_WAVES  // measurement build switch (-DKH_KEYS_WAVES=...): occupancy of key hashing
#define KH_KEYS_WAVES
#endif
// 32-bit sort word: the segment id in the top sb bits (segmented builds, sb <= CK_SEG_BITS),
// then the key's leading 32 - sb bits (big-endian)
__device__ __forceinline__ uint32_t ck_word(uint64_t h0, const uint32_t* seg, uint32_t sb, uint64_t i) {
  const uint32_t kb = (uint32_t)(bswap64(h0) >> 32);
  return sb ? (seg[i] << (32 - sb)) | (kb >> sb) : kb;
}
template <bool SHORT>
__global__ void __launch_bounds__(BS) KH_KEYS_WAVES k_hash_keys_ck(const uint8_t* keys, uint32_t klen, uint64_t first,
                                                                    uint64_t n, uint64_t* out, uint32_t* ck, uint32_t* idx,
                                                                    const uint32_t* seg, uint32_t sb) {
  // keys [first, n): one launch over all of them, or one per part of host inputs still arriving
  uint64_t i = first + (uint64_t)blockIdx.x * BS + threadIdx.x;
  if (i >= n) return;
  uint64_t h[4];
  if (SHORT)  // keys of <= 135 bytes (addresses, slot words): one block
    kec256_short(keys + i * klen, klen, h);
  else
    kec256_msg<false>(keys + i * klen, klen, h);
  for (int j = 0; j < 4; ++j) out[4 * i + j] = h[j];
  ck[i] = ck_word(h[0], seg, sb, i);
  idx[i] = (uint32_t)i;
}
// the same sort keys for caller-hashed keys
__global__ void __launch_bounds__(BS) k_make_ck32(const uint64_t* K, uint64_t n, uint32_t* ck, uint32_t* idx,
                                                  const uint32_t* seg, uint32_t sb) {
  uint64_t i = (uint64_t)blockIdx.x * BS + threadIdx.x;
  if (i >= n) return;
  ck[i] = ck_word(K[4 * i], seg, sb, i);
  idx[i] = (uint32_t)i;
}
// the sorted segment ids from the sorted 32-bit words (segmented ck path)
__global__ void __launch_bounds__(BS) k_sseg_from_ck(const uint32_t* sck, uint64_t m, uint32_t sb, uint32_t* sseg) {
  uint64_t i = (uint64_t)blockIdx.x * BS + threadIdx.x;
  if (i < m) sseg[i] = sb ? sck[i] >> (32 - sb) : 0u;  // sb = 0: one segment (a 32-bit shift would be undefined)
}

// composite sort key of key word 0 (k0): segment id in the top sb bits, then the key's leading
// bits (big-endian); flags |= 4 when the segment id needs more than sb bits
__device__ __forceinline__ uint64_t composite_ck(uint64_t k0, const uint32_t* seg, uint32_t sb, uint64_t i,
                                                 unsigned long long* flags) {
  const uint64_t be = bswap64(k0);
  if (!sb) return be;
  if (flags && sb < 32 && (seg[i] >> sb)) atomicOr(flags, 4ULL);
  return ((uint64_t)seg[i] << (64 - sb)) | (be >> sb);
}
// composite sort key: segment id in the top sb bits, then the key's leading bits (big-endian)
// (flags, nullable: |= 4 when a segment id needs more than sb bits -- a forest commit's sb is
// a hint from the trie ids seen before; the sort is then redone with 32)
// (rs_hdr, nullable: the radix sort's header zeroed here -- radix_sort_pairs then skips its fill
// launch; disjoint from everything else this kernel writes)
__global__ void __launch_bounds__(BS) k_make_ck(const uint64_t* K, const uint32_t* seg, uint32_t sb, uint64_t n,
                                                uint64_t* ck, uint32_t* idx, unsigned long long* flags,
                                                uint32_t* rs_hdr) {
  uint64_t i = (uint64_t)blockIdx.x * BS + threadIdx.x;
  if (rs_hdr)
    for (uint64_t w = i; w < RS_HDR_BYTES / 4; w += (uint64_t)gridDim.x * BS) rs_hdr[w] = 0;
  if (i >= n) return;
  ck[i] = composite_ck(K[4 * i], seg, sb, i, flags);
  idx[i] = (uint32_t)i;
}
// A forest commit's op keys after k_f_inputs (trie ids, counters zeroed, unhashed keys copied):
// the keys hashed (HASH: upserts then deletes), the composite sort keys made from them and the
// radix header zeroed -- one launch where two key-hashing launches and k_make_ck were
template <bool SHORT, bool HASH>
__global__ void __launch_bounds__(BS) k_f_keys_ck(const uint8_t* up_keys, uint64_t nup, const uint8_t* del_keys,
                                                  uint64_t ndel, uint32_t klen, uint64_t* K, const uint32_t* seg,
                                                  uint32_t sb, uint64_t* ck, uint32_t* idx, unsigned long long* flags,
                                                  uint32_t* rs_hdr) {
  const uint64_t o = (uint64_t)blockIdx.x * BS + threadIdx.x;
  for (uint64_t w = o; w < RS_HDR_BYTES / 4; w += (uint64_t)gridDim.x * BS) rs_hdr[w] = 0;
  if (o >= nup + ndel) return;
  uint64_t k0;
  if (HASH) {
    const uint8_t* key = o < nup ? up_keys + o * klen : del_keys + (o - nup) * klen;
    uint64_t h[4];
    if (SHORT)
      kec256_short(key, klen, h);
    else
      kec256_msg<false>(key, klen, h);
    for (int j = 0; j < 4; ++j) K[4 * o + j] = h[j];
    k0 = h[0];
  } else {
    k0 = K[4 * o];
  }
  ck[o] = composite_ck(k0, seg, sb, o, flags);
  idx[o] = (uint32_t)o;
}

// Runs of equal 32-bit sort prefixes (same segment, equal leading key bits) are
// put in full-key order by the thread at the run's start: an insertion sort of
// (key, index, segment) in place, stable, so among equal keys the input order
// (later put last) is kept.  flags |= 2 if equal keys exist (dedup needed; flags[-1]
// (CTR_NDUP) counts the keys dropped), |= 1 if a run exceeds TIE_RUN_MAX (take the
// full-sort path instead).
constexpr uint32_t TIE_RUN_MAX = 64;
// variable-length keys (zero padded, kn nibbles): a key sorts before the longer keys it
// prefixes, i.e. (padded key, length) order
__device__ __forceinline__ bool key_less(const uint64_t* a, const uint64_t* b, uint32_t kna = 0, uint32_t knb = 0) {
  for (int j = 0; j < 4; ++j) {
    uint64_t x = bswap64(a[j]), y = bswap64(b[j]);
    if (x != y) return x < y;
  }
  return kna < knb;
}
// (tsh: the composite prefixes were sorted on their bits from tsh up; a run is equal there)
__global__ void __launch_bounds__(BS) k_tie_fix(const uint64_t* ck, uint64_t n, uint64_t* skey, uint32_t* sidx,
                                                uint32_t* sseg, const uint8_t* kn, unsigned long long* flags,
                                                uint32_t tsh) {
  uint64_t i = (uint64_t)blockIdx.x * BS + threadIdx.x;
  if (i + 1 >= n) return;
  const uint64_t hi = ck[i] >> tsh;
  if ((ck[i + 1] >> tsh) != hi) return;   // no run starting or continuing here
  if (i > 0 && (ck[i - 1] >> tsh) == hi) return;  // not the run's first element
  uint64_t e = i + 1;
  while (e < n && (ck[e] >> tsh) == hi && e - i <= TIE_RUN_MAX) ++e;
  if (e - i > TIE_RUN_MAX) {
    atomicOr(flags, 1ULL);
    return;
  }
  for (uint64_t a = i + 1; a < e; ++a) {
    uint64_t k[4] = {skey[4 * a], skey[4 * a + 1], skey[4 * a + 2], skey[4 * a + 3]};
    uint32_t ix = sidx[a];
    uint32_t sg = sseg ? sseg[a] : 0;
    uint64_t b = a;
    const uint32_t kk = kn ? kn[ix] : 0;
    while (b > i && key_less(k, skey + 4 * (b - 1), kk, kn ? kn[sidx[b - 1]] : 0)) {
      for (int j = 0; j < 4; ++j) skey[4 * b + j] = skey[4 * (b - 1) + j];
      sidx[b] = sidx[b - 1];
      if (sseg) sseg[b] = sseg[b - 1];
      --b;
    }
    for (int j = 0; j < 4; ++j) skey[4 * b + j] = k[j];
    sidx[b] = ix;
    if (sseg) sseg[b] = sg;
  }
  unsigned long long ndup = 0;
  for (uint64_t a = i + 1; a < e; ++a) {
    const uint64_t* x = skey + 4 * (a - 1);
    const uint64_t* y = skey + 4 * a;
    ndup += (x[0] == y[0] && x[1] == y[1] && x[2] == y[2] && x[3] == y[3] && (!kn || kn[sidx[a - 1]] == kn[sidx[a]]))
                ? 1
                : 0;
  }
  if (ndup) {
    atomicOr(flags, 2ULL);
    atomicAdd(flags - 1, ndup);
  }
}

// Unsegmented plain builds sort (leading 32 key bits, index) pairs only; runs of equal
// prefixes are ordered here by the whole input key (through the index), stable; the keys
// themselves are never gathered into sorted order.
__device__ __forceinline__ bool ck_less(uint32_t a, uint32_t b, const uint64_t* K, uint32_t ia, uint32_t ib) {
  if (a != b) return a < b;
  return key_less(K + 4ull * ia, K + 4ull * ib);
}
__device__ __forceinline__ bool ck_equal(uint32_t a, uint32_t b, const uint64_t* K, uint32_t ia, uint32_t ib) {
  if (a != b) return false;
  const uint64_t* x = K + 4ull * ia;
  const uint64_t* y = K + 4ull * ib;
  return x[0] == y[0] && x[1] == y[1] && x[2] == y[2] && x[3] == y[3];
}
// the run of equal prefixes starting at i (ck[i] == ck[i + 1], i the run's first)
// u (nullable): also the boundary values inside the run, from the whole keys (k_lcp then
// skips boundaries between equal prefixes unless a dedup shifts the positions)
// (tsh 8: the words were sorted on their top 24 bits only; a run is equal there, its boundaries
// between different words valued here too -- from the whole keys, as lcp_value would)
__device__ void tie_run_ck(uint32_t* ck, uint32_t* idx, uint64_t n, const uint64_t* K, unsigned long long* flags,
                           uint64_t i, uint8_t* u = nullptr, uint32_t depth0 = 0, uint32_t tsh = 0) {
  const uint32_t hi = ck[i] >> tsh;
  uint64_t e = i + 1;
  while (e < n && (ck[e] >> tsh) == hi && e - i <= TIE_RUN_MAX) ++e;
  if (e - i > TIE_RUN_MAX) {
    atomicOr(flags, 1ULL);
    return;
  }
  for (uint64_t a = i + 1; a < e; ++a) {
    const uint32_t c = ck[a];
    const uint32_t ix = idx[a];
    uint64_t b = a;
    while (b > i && ck_less(c, ck[b - 1], K, ix, idx[b - 1])) {
      ck[b] = ck[b - 1];
      idx[b] = idx[b - 1];
      --b;
    }
    ck[b] = c;
    idx[b] = ix;
  }
  bool dup = false;
  for (uint64_t a = i + 1; a < e; ++a) dup |= ck_equal(ck[a - 1], ck[a], K, idx[a - 1], idx[a]);
  if (dup) atomicOr(flags, 2ULL);
  if (u)
    for (uint64_t a = i; a + 1 < e; ++a) {  // lcp_value's rule
      const int l = lcp_nibbles(load_key(K, idx[a]), load_key(K, idx[a + 1]));
      u[a] = (l < (int)depth0 || l > 63) ? 0 : (uint8_t)(l + 1);
    }
}
__device__ __forceinline__ bool tie_run_start(const uint32_t* ck, uint64_t n, uint64_t i) {
  if (i + 1 >= n) return false;
  const uint32_t hi = ck[i];
  return ck[i + 1] == hi && !(i > 0 && ck[i - 1] == hi);
}
// Block-local run list: a block covers TF_ITEMS * BS sorted positions, lists its run
// starts in LDS, and its first threads order the runs (wave 0 for the ~1 % of starting
// positions of random keys), so one wave per TF_ITEMS * 4 waves' worth of positions waits
// on a run's dependent key reads instead of nearly every wave (one thread per position).  A global list with one atomic per wave was
// measured far slower (a single contended counter: +9 ms at 100M).
constexpr int TF_ITEMS = 4;
// full_u (unsegmented words): the boundaries between different words are valued here too
// (lcp_value's rule from the words alone), so k_lcp does not read the words again
__global__ void __launch_bounds__(BS) k_tie_fix_ck_blk(uint32_t* ck, uint32_t* idx, uint64_t n, const uint64_t* K,
                                                       unsigned long long* flags, uint8_t* u, uint32_t depth0,
                                                       bool full_u, uint32_t tsh) {
  __shared__ uint32_t list[TF_ITEMS * BS];
  __shared__ uint32_t cnt;
  if (threadIdx.x == 0) cnt = 0;
  __syncthreads();
  const uint64_t base = (uint64_t)blockIdx.x * (TF_ITEMS * BS);
#pragma unroll
  for (int q = 0; q < TF_ITEMS; ++q) {
    const uint64_t i = base + (uint64_t)q * BS + threadIdx.x;
    if (i + 1 >= n) continue;
    const uint32_t a = ck[i], c = ck[i + 1];
    if ((a >> tsh) == (c >> tsh)) {
      if (!(i > 0 && (ck[i - 1] >> tsh) == (a >> tsh))) list[atomicAdd(&cnt, 1u)] = (uint32_t)(i - base);
    } else if (full_u) {
      const int l = (int)((uint32_t)clz64((uint64_t)(a ^ c) << 32) >> 2);
      u[i] = (l < (int)depth0 || l > 63) ? 0 : (uint8_t)(l + 1);
    }
  }
  __syncthreads();
  const uint32_t nr = cnt;
  for (uint32_t t = threadIdx.x; t < nr; t += BS) tie_run_ck(ck, idx, n, K, flags, base + list[t], u, depth0, tsh);
}

__global__ void __launch_bounds__(BS) k_dup_ck(const uint32_t* ck, const uint32_t* idx, const uint64_t* K, uint64_t n,
                                               uint32_t* keep) {
  uint64_t i = (uint64_t)blockIdx.x * BS + threadIdx.x;
  if (i >= n) return;
  keep[i] = (i + 1 < n && ck_equal(ck[i], ck[i + 1], K, idx[i], idx[i + 1])) ? 0u : 1u;
}
__global__ void __launch_bounds__(BS) k_compact_ck(const uint32_t* ck, const uint32_t* idx, const uint32_t* keep_pos,
                                                   const uint32_t* keep, uint64_t n, uint32_t* ock, uint32_t* oidx) {
  uint64_t i = (uint64_t)blockIdx.x * BS + threadIdx.x;
  if (i >= n || !keep[i]) return;
  const uint32_t p = keep_pos[i];
  ock[p] = ck[i];
  oidx[p] = idx[i];
}

// 32-byte keys move as two 16-byte vectors, both loads issued before any store
typedef uint64_t u64x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ void copy_key(const uint64_t* __restrict__ src, uint64_t* __restrict__ dst) {
  u64x2 a = ((const u64x2*)src)[0], b = ((const u64x2*)src)[1];
  ((u64x2*)dst)[0] = a;
  ((u64x2*)dst)[1] = b;
}

__global__ void __launch_bounds__(BS) k_gather(const uint64_t* __restrict__ K, const uint32_t* __restrict__ seg,
                                               const uint32_t* __restrict__ idx, uint64_t n,
                                               uint64_t* __restrict__ skey, uint32_t* __restrict__ sseg) {
  uint64_t i = (uint64_t)blockIdx.x * BS + threadIdx.x;
  if (i >= n) return;
  uint32_t s = idx[i];
  copy_key(K + 4 * (uint64_t)s, skey + 4 * i);
  if (seg) sseg[i] = seg[s];
}

__global__ void __launch_bounds__(BS) k_word_key(const uint64_t* K, const uint32_t* idx, int word, uint64_t n,
                                                 uint64_t* ck) {
  uint64_t i = (uint64_t)blockIdx.x * BS + threadIdx.x;
  if (i >= n) return;
  ck[i] = bswap64(K[4 * (uint64_t)idx[i] + word]);
}

__global__ void __launch_bounds__(BS) k_kn_key(const uint8_t* kn, const uint32_t* idx, uint64_t n, uint64_t* ck) {
  uint64_t i = (uint64_t)blockIdx.x * BS + threadIdx.x;
  if (i >= n) return;
  ck[i] = kn[idx[i]];
}
__global__ void __launch_bounds__(BS) k_kn_gather(const uint8_t* kn, const uint32_t* idx, uint64_t n, uint8_t* out) {
  uint64_t i = (uint64_t)blockIdx.x * BS + threadIdx.x;
  if (i < n) out[i] = kn[idx[i]];
}

__global__ void __launch_bounds__(BS) k_seg_key(const uint32_t* seg, const uint32_t* idx, uint64_t n, uint64_t* ck) {
  uint64_t i = (uint64_t)blockIdx.x * BS + threadIdx.x;
  if (i >= n) return;
  ck[i] = seg[idx[i]];
}

// keep the LAST of equal keys (later puts win, TrieAccounts.scala:23-27)
__global__ void __launch_bounds__(BS) k_dup(const uint64_t* skey, const uint32_t* sseg, const uint32_t* sidx,
                                            const uint8_t* kn, uint64_t n, uint32_t* keep) {
  uint64_t i = (uint64_t)blockIdx.x * BS + threadIdx.x;
  if (i >= n) return;
  uint32_t k = 1;
  if (i + 1 < n) {
    const uint64_t* a = skey + 4 * i;
    const uint64_t* b = a + 4;
    bool eq = a[0] == b[0] && a[1] == b[1] && a[2] == b[2] && a[3] == b[3];
    if (sseg && sseg[i] != sseg[i + 1]) eq = false;
    if (kn && kn[sidx[i]] != kn[sidx[i + 1]]) eq = false;
    k = eq ? 0 : 1;
  }
  keep[i] = k;
}

__global__ void __launch_bounds__(BS) k_compact(const uint64_t* skey, const uint32_t* sidx, const uint32_t* sseg,
                                                const uint32_t* keep_pos, const uint32_t* keep, uint64_t n,
                                                uint64_t* okey, uint32_t* oidx, uint32_t* oseg) {
  uint64_t i = (uint64_t)blockIdx.x * BS + threadIdx.x;
  if (i >= n || !keep[i]) return;
  uint64_t p = keep_pos[i];
  copy_key(skey + 4 * i, okey + 4 * p);
  oidx[p] = sidx[i];
  if (sseg) oseg[p] = sseg[i];
}

__global__ void __launch_bounds__(BS) k_val_gather(Topo T) {
  uint64_t i = (uint64_t)blockIdx.x * BS + threadIdx.x;
  if (i < T.m) op_val_gather(T, i);
}

// element builds: the element properties in sorted order
// element build: the value spans (op_val_gather) and both element property sets in sorted
// order, one launch
__global__ void __launch_bounds__(BS) k_el_gather3(Topo T, const uint8_t* db, const uint64_t* bref, const uint8_t* brl,
                                                   uint8_t* odb, uint64_t* obref, uint8_t* obrl, const uint8_t* db2,
                                                   const uint64_t* bref2, const uint8_t* brl2, uint8_t* odb2,
                                                   uint64_t* obref2, uint8_t* obrl2) {
  const uint64_t i = (uint64_t)blockIdx.x * BS + threadIdx.x;
  if (i >= T.m) return;
  op_val_gather(T, i);
  const uint32_t s = T.sidx[i];
  odb[i] = db[s];
  odb2[i] = db2[s];
  for (int q = 0; q < 4; ++q) {
    obref[4 * i + q] = bref[4ull * s + q];
    obref2[4 * i + q] = bref2[4ull * s + q];
  }
  obrl[i] = brl[s];
  obrl2[i] = brl2[s];
}

// ties_u: boundaries between equal 32-bit prefixes were valued by the tie-run kernel, unless
// a run was too long for it (tie flag bit 0: a speculative build, redone after its first sync
// with the full sort).  Such a run is left unordered and unvalued, so its boundaries get 0 (as
// between repeated keys: each key of the run a trie of its own) -- whatever the buffer held
// from an earlier build would shape a topology whose leaf depths leave 0..63.
// spec_clear: a speculative 64-bit composite sort (element builds) that met a run too long for the
// tie kernel left it unordered: every boundary 0 (each element a trie top; no branch) until the
// build is redone after its first sync
__global__ void __launch_bounds__(BS) k_lcp(Topo T, uint64_t nb, bool ties_u, const unsigned long long* tie,
                                            bool spec_clear, bool glast) {
  uint64_t b = (uint64_t)blockIdx.x * BS + threadIdx.x;
  if (b >= nb) return;
  if (glast) T.glast[b] = 1;  // (the whole-array topology's preset: no fill launch before it)
  if (spec_clear && (*tie & 1)) {
    T.u[b] = 0;
    return;
  }
  if (ties_u && T.sck[b] == T.sck[b + 1]) {
    if (*tie & 1) T.u[b] = 0;
    return;
  }
  op_lcp(T, b);
}
// every boundary was valued by the tie kernel: only a run too long for it (flag bit 0: a
// speculative build about to be redone) gets its boundaries cleared, as in k_lcp
__global__ void __launch_bounds__(BS) k_lcp_long_runs(Topo T, uint64_t nb, const unsigned long long* tie,
                                                      uint32_t tsh, bool glast) {
  const bool run = *tie & 1;
  if (!run && !glast) return;
  for (uint64_t b = (uint64_t)blockIdx.x * BS + threadIdx.x; b < nb; b += (uint64_t)gridDim.x * BS) {
    if (glast) T.glast[b] = 1;  // (the whole-array topology's preset: no fill launch before it)
    if (run && (T.sck[b] >> tsh) == (T.sck[b + 1] >> tsh)) T.u[b] = 0;
  }
}
// the 64-ary min pyramid over the boundary values: level `from` by the whole grid, the
// (small) upper levels by the last block to finish (the counter *done starts at zero;
// done == nullptr: level `from` only)
__global__ void __launch_bounds__(BS) k_pyramid(Pyr P, int from, unsigned int* done) {
  topo_prio();
  __shared__ bool last;
  const uint64_t i = (uint64_t)blockIdx.x * BS + threadIdx.x;
  if (i < P.sz[from]) op_min64(P.lv[from - 1], P.sz[from - 1], (uint8_t*)P.lv[from], i);
  if (!done) return;
  __threadfence();
  __syncthreads();
  if (threadIdx.x == 0) last = atomicAdd(done, 1u) == gridDim.x - 1;
  __syncthreads();
  if (!last) return;
  __threadfence();
  for (int l = from + 1; l < P.nl; ++l) {
    for (uint64_t k = threadIdx.x; k < P.sz[l]; k += BS) op_min64(P.lv[l - 1], P.sz[l - 1], (uint8_t*)P.lv[l], k);
    __threadfence_block();
    __syncthreads();
  }
}

__global__ void __launch_bounds__(BS) k_ansv(Topo T, Pyr P, uint64_t nb) {
  topo_prio();
  uint64_t b = (uint64_t)blockIdx.x * BS + threadIdx.x;
  if (b < nb) op_ansv(T, P, b);
}

// The topology kernels that run beside the leaf kernel are grid-stride loops, so their
// grid can be capped (topo_grid) to leave the leaf kernel more of the machine.
#define GRID_STRIDE(i, n) for (uint64_t i = (uint64_t)blockIdx.x * BS + threadIdx.x; i < (n); i += (uint64_t)gridDim.x * BS)
// the same with every thread of a block iterating together (i may pass n: wave-wide ballots)
#define GRID_STRIDE_WAVE(i, n)                                                                     \
  for (uint64_t i##_b = (uint64_t)blockIdx.x * BS, i = i##_b + threadIdx.x; i##_b < (n);        \
       i##_b += (uint64_t)gridDim.x * BS, i = i##_b + threadIdx.x)
__global__ void __launch_bounds__(BS) k_chain(Topo T, uint64_t nb) {
  topo_prio();
  GRID_STRIDE(b, nb) op_chain(T, b);
}
// ANSV and chains tile by tile in LDS (trie_ops.h op_tile_ansv / op_tile_chain), the boundaries
// whose answers leave the tile listed for k_ansv_list / k_chain_list; with pd, the early
// leaves' parent-depth scatter of the tile's sorted positions too (op_pd_scatter)
constexpr int TT_THREADS = 256;
// a tile's listed boundaries from its per-wave ballots (one 64-bit word per 64 boundaries):
// one wave, one global claim per list and tile
__device__ __forceinline__ void tile_list_out(const uint64_t* mask, uint64_t t0, unsigned long long* cnt, uint32_t* list) {
  const uint32_t lane = __lane_id();
  const uint64_t m = mask[lane];
  const uint32_t c = (uint32_t)__popcll(m);
  uint32_t x = c;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = __shfl_up(x, o);
    if ((int)lane >= o) x += y;
  }
  const uint32_t tot = __shfl(x, 63);
  if (tot == 0) return;
  unsigned long long base = 0;
  if (lane == 0) base = atomicAdd(cnt, (unsigned long long)tot);
  const uint32_t lo = (uint32_t)__shfl((int)(uint32_t)base, 0), hi = (uint32_t)__shfl((int)(uint32_t)(base >> 32), 0);
  uint64_t s = (((uint64_t)hi << 32) | lo) + (x - c);
  for (uint64_t r = m; r; r &= r - 1) list[s++] = (uint32_t)(t0 + 64 * lane + (uint32_t)__ffsll((long long)r) - 1);
}
__global__ void __launch_bounds__(TT_THREADS) k_topo_tile(Topo T, uint64_t nb, bool pd, unsigned long long* nlist,
                                                         uint32_t* alist, uint32_t* clist, uint8_t* pyr1) {
  __shared__ __align__(16) uint8_t su[TOPO_TILE + 16];
  __shared__ __align__(16) uint8_t sl1[64 + 16];
  __shared__ int16_t lpse[TOPO_TILE];
  __shared__ __align__(16) uint8_t lnext[TOPO_TILE];
  __shared__ uint8_t lrin[TOPO_TILE];
  __shared__ uint64_t amask[TOPO_TILE / 64], cmask[TOPO_TILE / 64];
  const uint64_t t0 = (uint64_t)blockIdx.x * TOPO_TILE;
  const uint32_t tn = (uint32_t)(nb - t0 < TOPO_TILE ? nb - t0 : TOPO_TILE);
  // the presets two fills wrote before this kernel (a fill launch each on the critical path):
  // glast 1 over the tile's boundaries (whole 16-byte words; this block's phase 1 clears some,
  // after the barrier below), lf_emeta 32 over its sorted leaves (the last tile: through m - 1)
  {
    const uint64_t gend = t0 + ((tn + 15) & ~15u);
    const uint64_t lend = blockIdx.x + 1 == gridDim.x ? (pd ? T.m : t0) : t0 + TOPO_TILE;
    const ulonglong2 ones{0x0101010101010101ULL, 0x0101010101010101ULL};
    for (uint64_t o = t0 + 16 * threadIdx.x; o < gend; o += 16 * TT_THREADS) *(ulonglong2*)(T.glast + o) = ones;
    if (pd)
      for (uint64_t o = t0 + threadIdx.x; o < lend; o += TT_THREADS) T.lf_emeta[o] = 32;
  }
  for (uint32_t w = threadIdx.x; w < TOPO_TILE / 16; w += TT_THREADS) {
    const uint32_t o = 16 * w;
    if (o + 16 <= tn) {
      *(ulonglong2*)(su + o) = *(const ulonglong2*)(T.u + t0 + o);  // (u is carved 256-byte aligned)
    } else {
      for (uint32_t q = 0; q < 16; ++q) su[o + q] = o + q < tn ? T.u[t0 + o + q] : (uint8_t)0x7F;
    }
    *(ulonglong2*)(lnext + o) = ulonglong2{0, 0};
  }
  __syncthreads();
  if (threadIdx.x < 64) {
    uint32_t mn = 0x7F;
    for (uint32_t q = 0; q < 64; ++q) mn = min(mn, (uint32_t)su[64 * threadIdx.x + q]);
    sl1[threadIdx.x] = (uint8_t)mn;
    // the whole-array pyramid's first level is these minima (op_min64 over the same 64 values;
    // past nb the tile holds 0x7F, above every boundary value): k_pyramid starts one level up
    if (pyr1 && 64 * threadIdx.x < tn) pyr1[t0 / 64 + threadIdx.x] = (uint8_t)mn;
  }
  __syncthreads();
  const TilePyr P{su, sl1, tn, (tn + 63) / 64};
  const uint32_t wv = threadIdx.x >> 6;
  for (uint32_t k = 0; k < TOPO_TILE / TT_THREADS; ++k) {
    const uint32_t i = k * TT_THREADS + threadIdx.x;
    const uint64_t m = __ballot(i < tn && op_tile_ansv(T, P, t0, i, lpse, lnext, lrin));
    if (__lane_id() == 0) amask[k * (TT_THREADS / 64) + wv] = m;
  }
  __syncthreads();
  for (uint32_t k = 0; k < TOPO_TILE / TT_THREADS; ++k) {
    const uint32_t i = k * TT_THREADS + threadIdx.x;
    uint32_t isr = 0;
    const uint64_t m = __ballot(i < tn && op_tile_chain(T, P, t0, i, lpse, lnext, lrin, &isr));
    if (__lane_id() == 0) cmask[k * (TT_THREADS / 64) + wv] = m;
    if (T.rep_bits) {  // the wave's 64 boundaries' representative flags: two bit words (every word of
                       // the tile written; k_chain_list ORs in the listed boundaries' flags after it)
      const uint64_t rb = __ballot(isr != 0);
      if (__lane_id() == 0) *(uint64_t*)(T.rep_bits + ((t0 + k * TT_THREADS + 64 * wv) >> 5)) = rb;
    }
  }
  __syncthreads();
  if (wv == 0) tile_list_out(amask, t0, &nlist[0], alist);
  if (wv == 1) tile_list_out(cmask, t0, &nlist[1], clist);
  if (pd) {  // sorted leaves [t0, t0 + TOPO_TILE) (the last tile: through m - 1 = nb)
    const uint64_t lend = blockIdx.x + 1 == gridDim.x ? T.m : t0 + TOPO_TILE;
    for (uint64_t i = t0 + threadIdx.x; i < lend; i += TT_THREADS) {  // (the tile's values from LDS)
      const uint32_t q = (uint32_t)(i - t0);
      pd_scatter_vals(T, i, q > 0 ? su[q - 1] : i > 0 ? T.u[i - 1] : 0, q < tn ? su[q] : 0);
    }
  }
}
// the listed boundaries (grid-stride over the device's list count)
__global__ void __launch_bounds__(BS) k_ansv_list(Topo T, Pyr P, const uint32_t* list, const unsigned long long* cnt) {
  topo_prio();
  const uint64_t n = *cnt;
  for (uint64_t i = (uint64_t)blockIdx.x * BS + threadIdx.x; i < n; i += (uint64_t)gridDim.x * BS) op_ansv(T, P, list[i]);
}
__global__ void __launch_bounds__(BS) k_chain_list(Topo T, const uint32_t* list, const unsigned long long* cnt) {
  topo_prio();
  const uint64_t n = *cnt;
  for (uint64_t i = (uint64_t)blockIdx.x * BS + threadIdx.x; i < n; i += (uint64_t)gridDim.x * BS) op_chain(T, list[i]);
}
// k_ansv with the early leaves' parent-depth scatter folded in (thread i also scatters
// leaf i; grid over the m leaves): the leaf kernel waits for this kernel instead of a
// separate k_pd_scatter racing the topology for the memory system (run_build)
__global__ void __launch_bounds__(BS) k_ansv_pd(Topo T, Pyr P, uint64_t nb) {
  uint64_t b = (uint64_t)blockIdx.x * BS + threadIdx.x;
  if (b < nb) op_ansv(T, P, b);
  if (b < T.m) op_pd_scatter(T, b);
}

// sum three per-thread counters over the block; one atomic per counter per block
__device__ __forceinline__ void block_add3(unsigned long long* c0, unsigned long long v0, unsigned long long* c1,
                                           unsigned long long v1, unsigned long long* c2, unsigned long long v2) {
  __shared__ unsigned long long red[BS / 64][3];
  v0 = wave_sum(v0);
  v1 = wave_sum(v1);
  v2 = wave_sum(v2);
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    red[w][0] = v0;
    red[w][1] = v1;
    red[w][2] = v2;
  }
  __syncthreads();
  if (threadIdx.x < 3) {
    unsigned long long t = 0;
    for (int q = 0; q < BS / 64; ++q) t += red[q][threadIdx.x];
    unsigned long long* dst = threadIdx.x == 0 ? c0 : threadIdx.x == 1 ? c1 : c2;
    if (t && dst) atomicAdd(dst, t);
  }
}

__global__ void __launch_bounds__(BS) k_branch_topo(Topo T, Pyr P, uint64_t nb) {
  topo_prio();
  unsigned long long ext = 0;
  GRID_STRIDE(b, nb) ext += op_branch_topo(T, P, nb, b);
  block_add3(ctr_stat(T.ctr, CTR_EXT, blockIdx.x), ext, nullptr, 0, nullptr, 0);
}

__global__ void __launch_bounds__(BS) k_leaf_topo(Topo T) {
  uint64_t i = (uint64_t)blockIdx.x * BS + threadIdx.x;
  if (i < T.m)
    op_leaf_topo(T, i, [&](uint64_t b) { return (uint64_t)atomicAdd(&T.ctr[CTR_LFBYTES], (unsigned long long)b); });
}

// Level order without contended global atomics: branch ids bucketed by
//   bucket = depth * 8 + has_extension * 4 + (3 - (blocks - 1))
// (blocks = Keccak blocks of the branch if every child is hashed), so a level is
// the contiguous range of its 8 buckets, heaviest branches first and extensions
// grouped: the waves of a level run the same number of permutations.  Per-block
// bucket counts are laid out [bucket][block]; one exclusive scan gives every
// (bucket, block) its base; a second pass ranks inside the block with LDS atomics.
// (Bucketed by the exact child count instead -- waves with uniform child loops -- the
// children ranges of neighbouring branches are no longer adjacent: depth 6 5.06 -> 5.32 ms,
// 11.8 -> 14.5 GB read, profiles/r5m_level_order_ab_100m.json.)
constexpr uint32_t LV_PER_DEPTH = 8;
constexpr uint32_t NBUCKET = 64 * LV_PER_DEPTH;
__device__ __forceinline__ uint32_t branch_bucket(const Topo& T, uint64_t j) {
  uint32_t k = T.br_k[j];
  uint32_t payload = 32 * k + 17;
  uint32_t blocks = perms_for_len(rlp_hdr_len(payload) + payload);  // 1..4
  return (uint32_t)T.br_depth[j] * 8 + (T.br_ext[j] ? 4 : 0) + (4 - blocks);
}
constexpr uint32_t LV_IT = 16;          // branch ids per thread
constexpr uint32_t LV_TILE = BS * LV_IT;  // branch ids per block: few blocks -> a short [bucket][block] table
// the buckets of a thread's LV_IT branch ids, their loads issued together (one round trip, not
// LV_IT dependent ones: a block commit's element builds are latency-bound); NBUCKET past B
__device__ __forceinline__ void level_buckets(const Topo& T, uint64_t B, uint32_t (&bk)[LV_IT]) {
  const uint64_t j0 = (uint64_t)blockIdx.x * LV_TILE + threadIdx.x;
#pragma unroll
  for (uint32_t q = 0; q < LV_IT; ++q) {
    const uint64_t j = j0 + (uint64_t)q * BS;
    bk[q] = j < B ? branch_bucket(T, j) : NBUCKET;
  }
}
// The table's stride is the device's block count for the B branches, ceil(B / LV_TILE): the grid
// is sized by the boundaries (B is not on the host yet), and a 100M build's B is a third of them --
// the blocks past it neither write nor are scanned (the [bucket][block] stores are scattered:
// 32-byte sectors for 4-byte counts, 0.4 GB a 100M build with the host's bound)
__device__ __forceinline__ uint32_t level_blocks(const uint32_t* Bp) {
  return (uint32_t)(((uint64_t)*Bp + LV_TILE - 1) / LV_TILE);
}
__global__ void __launch_bounds__(BS) k_level_count(Topo T, const uint32_t* Bp, uint32_t* bcnt, uint32_t* ncnt) {
  topo_prio();
  const uint32_t nblk = level_blocks(Bp);
  if (blockIdx.x == 0 && threadIdx.x == 0) *ncnt = NBUCKET * nblk;  // (the table scan's count)
  if (blockIdx.x >= nblk) return;
  __shared__ uint32_t h[NBUCKET];
  for (uint32_t q = threadIdx.x; q < NBUCKET; q += BS) h[q] = 0;
  uint32_t bk[LV_IT];
  level_buckets(T, *Bp, bk);
  __syncthreads();
#pragma unroll
  for (uint32_t q = 0; q < LV_IT; ++q)
    if (bk[q] < NBUCKET) atomicAdd(&h[bk[q]], 1u);
  __syncthreads();
  for (uint32_t q = threadIdx.x; q < NBUCKET; q += BS) bcnt[(uint64_t)q * nblk + blockIdx.x] = h[q];
}

// pos[j] = position of branch j (numbered in key order by the rep scan) in the
// level order; the branch tables are then permuted to that order (k_branch_permute)
// so a level reads its branches' fields, child records and message slots contiguously
__global__ void __launch_bounds__(BS) k_level_scatter(Topo T, const uint32_t* Bp, const uint32_t* bbase,
                                                      uint32_t* pos) {
  topo_prio();
  const uint32_t nblk = level_blocks(Bp);
  if (blockIdx.x >= nblk) return;
  __shared__ uint32_t base[NBUCKET];
  for (uint32_t q = threadIdx.x; q < NBUCKET; q += BS) base[q] = bbase[(uint64_t)q * nblk + blockIdx.x];
  uint32_t bk[LV_IT];
  level_buckets(T, *Bp, bk);
  __syncthreads();
  const uint64_t j0 = (uint64_t)blockIdx.x * LV_TILE + threadIdx.x;
#pragma unroll
  for (uint32_t q = 0; q < LV_IT; ++q)
    if (bk[q] < NBUCKET) pos[j0 + (uint64_t)q * BS] = atomicAdd(&base[bk[q]], 1u);
}

// the branch tables k_branch_topo wrote in key-order ids (J), moved to level order
struct BrTab {
  uint32_t *k, *parent, *first, *end;  // (end: leaf positions only)
  uint8_t *depth, *ext, *pord;
};
__global__ void __launch_bounds__(BS) k_branch_permute(Topo T, BrTab J, const uint32_t* pos, const uint32_t* Bp) {
  topo_prio();
  const uint64_t B = *Bp;
  GRID_STRIDE(j, B) {
    const uint32_t g = pos[j], p = J.parent[j];
    T.br_k[g] = J.k[j];
    T.br_depth[g] = J.depth[j];
    T.br_ext[g] = J.ext[j];
    T.br_pord[g] = J.pord[j];
    T.br_first[g] = J.first[j];
    if (T.br_end) T.br_end[g] = J.end[j];
    T.br_parent[g] = p == NONE ? NONE : pos[p];  // parents of neighbouring branches are neighbours
  }
}
// rep_pref[w] = popcount of the representative bit word w (scanned in place afterwards)
__global__ void __launch_bounds__(BS) k_rep_popc(const uint32_t* bits, uint64_t nw, uint32_t* pref) {
  topo_prio();
  GRID_STRIDE(w, nw) pref[w] = (uint32_t)__popc(bits[w]);
}
// group reps carry level-order branch ids from here on (leaf parents, resident tables)
__global__ void __launch_bounds__(BS) k_bid_remap(Topo T, const uint32_t* pos, uint64_t nb) {
  topo_prio();
  GRID_STRIDE(b, nb) if (T.u[b] != 0 && T.rep[b] == (uint32_t)b) T.isrep_bid[b] = pos[T.isrep_bid[b]];
}

// level bounds: lb[d] = first position of depth d in `order`, lb[64] = B
__global__ void k_level_bounds(const uint32_t* bbase, const uint32_t* Bp, uint32_t* lb) {
  topo_prio();
  const uint32_t nblk = level_blocks(Bp);
  uint32_t d = threadIdx.x;
  if (d < 64) lb[d] = nblk ? bbase[(uint64_t)d * LV_PER_DEPTH * nblk] : 0;
  if (d == 0) lb[64] = *Bp;
}

// Leaf encode.  The value spans are random in the input buffer; if every lane
// walked its own span with 8-byte loads, the ~12 dependent loads per lane would be
// spread over time and the lines re-fetched after L2 eviction (measured ~570 B of
// fabric reads per 80 B value).  Instead each wave first copies the spans of its 64
// leaves into LDS cooperatively (16 lanes per span, one coalesced 128 B request),
// then every lane encodes its own leaf from LDS.  Spans wider than the stage are
// read from global memory directly (long values; such leaves go to the arena).
constexpr uint32_t STAGE_WORDS = 19;  // aligned 8-byte words per staged value span

// Slots for a whole block at once: one atomic per block (the gather's per-wave claims on the
// one element counter serialised in L2).  Every thread of the block must call it.
__device__ __forceinline__ uint64_t block_claim(unsigned long long* ctr, bool want, unsigned long long* lds) {
  const uint64_t m = __ballot(want);
  const uint32_t w = threadIdx.x >> 6, nw = blockDim.x >> 6;
  if ((threadIdx.x & 63) == 0) lds[w] = (unsigned long long)__popcll(m);
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned long long run = 0;
    for (uint32_t q = 0; q < nw; ++q) {
      const unsigned long long c = lds[q];
      lds[q] = run;
      run += c;
    }
    lds[nw] = run ? atomicAdd(ctr, run) : 0;
  }
  __syncthreads();
  const uint64_t e = lds[nw] + lds[w] + (uint64_t)__popcll(m & lanemask_lt());
  __syncthreads();  // lds is reused by the next call
  return e;
}
// Element builds (a block commit): most elements are unchanged subtrees or leaves whose
// reference is only handed to the new parent; the few that are re-encoded (the block's
// upserts, moved leaves, new extensions) sit scattered among them, so a thread-per-element
// hash pass runs a permutation in nearly every wave.  k_leaf_prep publishes the cheap ones
// and lists the others (one claim per block); k_leaf_hash_list hashes the list in full waves.
__device__ __forceinline__ bool leaf_listed(const Topo& T, uint64_t i) {
  if (is_branch_value(T, i)) return false;
  const uint32_t a = (uint32_t)(T.lf_pd[i] + 1);
  return !(el_cached(T, i, a) || (el_subtree(T, i) && el_ext_nibbles(T, i, a) == 0));
}
// pass (element builds with late values, ElemArgs::late): 0 every element; 1 all but the late
// ones (before their values arrive); 2 only the late ones
// pass 0: every element; 1: those whose value is not late, the late ones listed into (late,
// *nlate); 2: the listed late ones only (thread t: late[t]), each hashed here rather than
// listed for k_leaf_hash_list -- the late values arrive last, and a pass over every element
// plus a hash launch after them was ~60 us on the block commit's critical path
__global__ void __launch_bounds__(BS) k_leaf_prep(Topo T, uint32_t* list, unsigned long long* nlist, int pass,
                                                  uint32_t* late, unsigned long long* nlate) {
  __shared__ uint64_t stage[BS * STAGE_WORDS];
  __shared__ unsigned long long claim[BS / 64 + 1], claim2[BS / 64 + 1];
  uint64_t i = (uint64_t)blockIdx.x * BS + threadIdx.x;
  if (pass == 2) {
    const uint64_t nl = *nlate;
    if ((uint64_t)blockIdx.x * BS >= nl) return;  // (block-uniform)
    i = i < nl ? late[i] : T.m;
  }
  bool mine = i < T.m;
  if (pass == 1) {
    const bool is_late = mine && T.el_late[T.sidx[i]] != 0;
    const uint64_t e = block_claim(nlate, is_late, claim2);
    if (is_late) late[e] = (uint32_t)i;
    mine = mine && !is_late;
  }
  const uint32_t ln = threadIdx.x & 63, wbase = threadIdx.x & ~63u;
  uint64_t off = 0;
  uint32_t vlen = 0;
  // (an element build's cached nodes and subtrees are not re-encoded: their values are not
  // staged -- most elements of a block commit, the unchanged siblings on the dirty paths)
  if (mine && !(T.el_db && (el_subtree(T, i) || el_cached(T, i, (uint32_t)(T.lf_pd[i] + 1))))) {
    off = T.svoff[i];
    vlen = T.svlen[i];
  }
  const uint32_t vmis = (uint32_t)((uintptr_t)T.vals & 7);  // vals base misalignment
  typedef const __attribute__((address_space(1))) uint64_t gword;  // global (not flat) loads
  gword* vw = (gword*)(T.vals - vmis);
  const uint64_t a0 = (off + vmis) >> 3;                     // first aligned word of the span
  const uint32_t nw = vlen ? (uint32_t)(((off + vmis + vlen + 7) >> 3) - a0) : 0;
  const uint32_t g = ln >> 4, gl = ln & 15;
  // four spans' loads issued together, then their LDS stores (per-span conditions around each
  // load made every one of a wave's 32 loads a round trip of its own: the latency-bound passes --
  // a block commit's late leaves -- spent ~50 us there); a lane with nothing to load reads the
  // values' first word instead (unused)
  if (T.vals) {
#pragma unroll
    for (uint32_t it0 = 0; it0 < 16; it0 += 4) {
      uint64_t w0[4], w1[4];
      uint32_t sn[4];
      uint64_t sa[4];
#pragma unroll
      for (uint32_t q = 0; q < 4; ++q) {
        const uint32_t src = (it0 + q) * 4 + g;  // lane of the wave whose span this group copies
        sa[q] = __shfl(a0, (int)src);
        const uint32_t n = __shfl(nw, (int)src);
        sn[q] = n <= STAGE_WORDS ? n : 0;
      }
      // (the wave's 16 spans here all empty -- cached elements and subtrees, most of a block
      // commit's: no loads)
      if (!__ballot((sn[0] | sn[1] | sn[2] | sn[3]) != 0)) continue;
#pragma unroll
      for (uint32_t q = 0; q < 4; ++q) {
        w0[q] = vw[gl < sn[q] ? sa[q] + gl : 0];
        w1[q] = vw[gl + 16 < sn[q] ? sa[q] + gl + 16 : 0];
      }
#pragma unroll
      for (uint32_t q = 0; q < 4; ++q) {
        uint64_t* dst = stage + (wbase + (it0 + q) * 4 + g) * STAGE_WORDS;
        if (gl < sn[q]) dst[gl] = w0[q];
        if (gl + 16 < sn[q]) dst[gl + 16] = w1[q];
      }
    }
  }
  __syncthreads();
  if (mine) {
    if (nw <= STAGE_WORDS)  // two call sites so each keeps its address space (ds_read vs global_load)
      op_leaf_prep(T, i, (const uint8_t*)(stage + threadIdx.x * STAGE_WORDS) + ((off + vmis) & 7), vlen);
    else
      op_leaf_prep(T, i, T.vals + off, vlen);
  }
  if (!list) return;  // (block-uniform) element builds: publish the kept references, list the rest
  const bool live = mine;
  const bool listed = live && pass != 2 && leaf_listed(T, i);
  unsigned long long perms = 0, hashes = 0, inl = 0;
  if (live && !listed) {
    uint32_t in1 = 0;
    perms = op_leaf_hash(T, i, &in1);
    hashes = perms ? 1 : 0;
    inl = in1;
  }
  const uint64_t e = block_claim(nlist, listed, claim);
  if (listed) list[e] = (uint32_t)i;
  block_add3(ctr_stat(T.ctr, CTR_PERMS, blockIdx.x), perms, ctr_stat(T.ctr, CTR_HASHES, blockIdx.x), hashes,
             ctr_stat(T.ctr, CTR_INLINE, blockIdx.x), inl);
}

__global__ void __launch_bounds__(BS) k_leaf_hash(Topo T) {
  uint64_t i = (uint64_t)blockIdx.x * BS + threadIdx.x;
  unsigned long long perms = 0, hashes = 0, inl = 0;
  if (i < T.m) {
    uint32_t in1 = 0;
    perms = op_leaf_hash(T, i, &in1);
    hashes = perms ? 1 : 0;
    inl = in1;
  }
  block_add3(ctr_stat(T.ctr, CTR_PERMS, blockIdx.x), perms, ctr_stat(T.ctr, CTR_HASHES, blockIdx.x), hashes,
             ctr_stat(T.ctr, CTR_INLINE, blockIdx.x), inl);
}
__global__ void __launch_bounds__(BS) k_leaf_hash_list(Topo T, const uint32_t* list, const unsigned long long* nlist) {
  const uint64_t n = *nlist;
  unsigned long long perms = 0, hashes = 0, inl = 0;
  for (uint64_t k = (uint64_t)blockIdx.x * BS + threadIdx.x; k < n; k += (uint64_t)gridDim.x * BS) {
    uint32_t in1 = 0;
    const uint32_t p = op_leaf_hash(T, list[k], &in1);
    perms += p;
    hashes += p ? 1 : 0;
    inl += in1;
  }
  block_add3(ctr_stat(T.ctr, CTR_PERMS, blockIdx.x), perms, ctr_stat(T.ctr, CTR_HASHES, blockIdx.x), hashes,
             ctr_stat(T.ctr, CTR_INLINE, blockIdx.x), inl);
}

// the early leaves' parent depths and sorted positions for a trie too small for a topology
// (one key: no boundaries, no ANSV to fold the scatter into)
__global__ void __launch_bounds__(BS) k_pd_scatter(Topo T) {
  uint64_t i = (uint64_t)blockIdx.x * BS + threadIdx.x;
  if (i < T.m) op_pd_scatter(T, i);
}
// per-wave counter add: the lanes' flags counted by ballot, one atomic per wave
__device__ __forceinline__ void wave_count(unsigned long long* dst, bool f) {
  const uint64_t b = __ballot(f);
  if (b && __lane_id() == 0) atomicAdd(dst, (unsigned long long)__popcll(b));
}
// Early leaves: k_leaf_in (csrc/leaf_kernel.hip, a compilation unit of its own: see there)
constexpr uint32_t LEAF_ITEMS = 4;  // runs of BS inputs per block (leaf_kernel.hip)
__global__ void k_leaf_in(Topo T, uint64_t n);
// the same publish split in two (trie_ops.h op_leaf_link / op_leaf_move)
__global__ void __launch_bounds__(BS) k_leaf_link(Topo T) {
  GRID_STRIDE(i, T.m) op_leaf_link(T, i);
}
// after the join (leaf positions): the long leaves' arena slots and parents
// (op_leaf_topo_early), for k_leaf_long
__global__ void __launch_bounds__(BS) k_leaf_fix(Topo T, uint64_t nlong) {
  const uint64_t q = (uint64_t)blockIdx.x * BS + threadIdx.x;
  if (q < nlong)
    op_leaf_topo_early(T, T.longlist[q],
                       [&](uint64_t b) { return (uint64_t)atomicAdd(&T.ctr[CTR_LFBYTES], (unsigned long long)b); });
}
__global__ void __launch_bounds__(BS) k_leaf_move(Topo T) {
  uint64_t i = (uint64_t)blockIdx.x * BS + threadIdx.x;
  if (i < T.m)
    op_leaf_move(T, i, [&](uint64_t b) { return (uint64_t)atomicAdd(&T.ctr[CTR_LFBYTES], (unsigned long long)b); });
}

__global__ void __launch_bounds__(BS) k_leaf_long(Topo T) {
  uint64_t i = (uint64_t)blockIdx.x * BS + threadIdx.x;
  unsigned long long perms = 0, hashes = 0, inl = 0;
  if (i < T.m) {
    uint32_t in1 = 0;
    perms = op_leaf_long(T, i, &in1);
    hashes = perms ? 1 : 0;
    inl = in1;
  }
  block_add3(ctr_stat(T.ctr, CTR_PERMS, blockIdx.x), perms, ctr_stat(T.ctr, CTR_HASHES, blockIdx.x), hashes,
             ctr_stat(T.ctr, CTR_INLINE, blockIdx.x), inl);
}

// one level: `first` = its first position in the level order, `cnt` = its size;
// branch ids are level positions (k_branch_permute)
__global__ void __launch_bounds__(BS) k_branch_prep(Topo T, uint64_t first, uint64_t cnt) {
  uint64_t t = (uint64_t)blockIdx.x * BS + threadIdx.x;
  if (t < cnt) op_branch_prep(T, (uint32_t)(first + t), first + t);
}

__global__ void __launch_bounds__(BS) k_branch_hash(Topo T, uint64_t first, uint64_t cnt) {
  uint64_t t = (uint64_t)blockIdx.x * BS + threadIdx.x;
  unsigned long long perms = 0, hashes = 0, inl = 0;
  if (t < cnt) {
    uint32_t j = (uint32_t)(first + t);
    uint32_t in1 = 0;
    perms = op_branch_hash(T, j, first + t, &in1);
    hashes = branch_hash_count(T, j, (uint32_t)perms);
    inl = in1;
  }
  block_add3(ctr_stat(T.ctr, CTR_PERMS, blockIdx.x), perms, ctr_stat(T.ctr, CTR_HASHES, blockIdx.x), hashes,
             ctr_stat(T.ctr, CTR_INLINE, blockIdx.x), inl);
}

// Fused per-level branch kernel (root-only and incremental builds; row N1): each thread
// streams its branch's encoding block by block through its own 17-word LDS slot into
// the Keccak state (op_branch_fused), so no branch RLP is written to or read back from
// HBM: the level reads its contiguous child records once and writes one 34-byte
// reference per node.  Slot layout [thread][word]: a wave's 8-byte slot accesses are
// bank-conflict-free within each 16-lane group (stride 34 dwords).
// V: 0 variable-length keys (op_branch_fused), 2 the children streamed once with the next
// record prefetched (op_branch_stream), 4 the same reading leaf children at their sorted
// positions (leaf positions) through the 12-bit child table (SRC_T12: the children's metas
// loaded in one round; a wave with a branch spanning 4096+ keys takes SRC_POS), 6 the same
// below depth 8 (the nibble from the input key).  Child table vs metas loaded child by child:
// branch levels 7.91-7.95 -> 7.85-7.87 ms, reads 21.0 -> 16.3 GB at 100M
// (profiles/r5u_branch_table12_ab_100m.json); one more child in flight spills 19 VGPRs and
// costs 0.5 ms (r5v_branch_table12_queue_ab_100m.json).
// V 4 / 6 take the table form only: a branch spanning T12_SPAN keys or more (rare: the top of
// a trie, a cluster of keys) is listed for k_branch_wide, launched right after on the level.
// With both forms in one kernel its registers were the larger form's: 128 VGPRs with 10
// spilled to scratch (the addresses of the branch's own table entries, reloaded ~11 times
// a thread); the table form alone fits in 127 with none.
template <int V>
__global__ void __launch_bounds__(BS) __attribute__((amdgpu_waves_per_eu(4, 8))) k_branch_fused(Topo T, uint64_t first, uint64_t cnt) {
  __shared__ uint64_t slots[BS * LEAF_WORDS];
  constexpr bool TB = V == 4 || V == 6;
  __shared__ uint32_t tbl[TB ? 6 * BS : 1];  // [dword][thread]: 24 B per lane beside its 136-byte window
  uint64_t t = (uint64_t)blockIdx.x * BS + threadIdx.x;
  unsigned long long perms = 0, hashes = 0, inl = 0;
  if (t < cnt) {
    uint32_t j = (uint32_t)(first + t);
    uint32_t in1 = 0;
    // fixed-length keys: direct window assembly; variable-length keys (branch values):
    // the byte stream through the windowed writer
    uint64_t* sl = slots + threadIdx.x * LEAF_WORDS;
    const bool wide = TB && T.br_end[j] - T.br_first[j] >= T12_SPAN;
    const ChildSrc ts{nullptr, nullptr, 1, tbl + threadIdx.x, BS};
    if (wide) {
      T.wlist[atomicAdd(T.wcnt, 1u)] = j;
    } else {
      perms = V == 0   ? op_branch_fused(T, j, sl, 1, &in1)
              : V == 2 ? op_branch_stream_t<SRC_REC>(T, j, sl, 1, &in1, ChildSrc{})
              : V == 4 ? op_branch_stream_t<SRC_T12>(T, j, sl, 1, &in1, ts)
                       : op_branch_stream_t<SRC_T12K>(T, j, sl, 1, &in1, ts);
      hashes = branch_hash_count(T, opaque_u32(j), (uint32_t)perms);
      inl = in1;
    }
  }
  // one atomic per wave (a block-wide sum would need LDS past the 40 KB that 4 blocks per CU allow)
  const unsigned long long sp = wave_sum(perms), sh = wave_sum(hashes), si = wave_sum(inl);
  if ((threadIdx.x & 63) == 0) {
    if (sp) atomicAdd(ctr_stat(T.ctr, CTR_PERMS, blockIdx.x), sp);
    if (sh) atomicAdd(ctr_stat(T.ctr, CTR_HASHES, blockIdx.x), sh);
    if (si) atomicAdd(ctr_stat(T.ctr, CTR_INLINE, blockIdx.x), si);
  }
}

// The branches k_branch_fused<4 / 6> listed (spanning T12_SPAN keys or more): the per-child
// form (every child's meta loaded as its record is placed).  Usually none at the big levels of
// random keys: a few blocks that read the count and exit.
template <int V>
__global__ void __launch_bounds__(BS) k_branch_wide(Topo T) {
  __shared__ uint64_t slots[BS * LEAF_WORDS];
  const uint32_t nw = *(volatile const uint32_t*)T.wcnt;
  unsigned long long perms = 0, hashes = 0, inl = 0;
  for (uint32_t t = blockIdx.x * BS + threadIdx.x; t < nw; t += gridDim.x * BS) {
    const uint32_t j = T.wlist[t];
    uint32_t in1 = 0;
    uint64_t* sl = slots + threadIdx.x * LEAF_WORDS;
    const uint32_t p = V == 4 ? op_branch_stream_t<SRC_POS>(T, j, sl, 1, &in1, ChildSrc{})
                              : op_branch_stream_t<SRC_POSK>(T, j, sl, 1, &in1, ChildSrc{});
    perms += p;
    hashes += branch_hash_count(T, j, p);
    inl += in1;
  }
  const unsigned long long sp = wave_sum(perms), sh = wave_sum(hashes), si = wave_sum(inl);
  if ((threadIdx.x & 63) == 0) {
    if (sp) atomicAdd(ctr_stat(T.ctr, CTR_PERMS, blockIdx.x), sp);
    if (sh) atomicAdd(ctr_stat(T.ctr, CTR_HASHES, blockIdx.x), sh);
    if (si) atomicAdd(ctr_stat(T.ctr, CTR_INLINE, blockIdx.x), si);
  }
}

// Small levels (a block commit's dirty paths, the few branches at the top of a full build):
// latency-bound, a wave or less per CU.  op_branch_stream prefetches one child record
// ahead, so a full branch waits for 16 HBM round trips in a row.  Here every child record
// of the branch is loaded at once (16 x 32 B in flight per thread) and copied to LDS
// (lane-interleaved, conflict-free), and the stream reads it from there.  A lane pair per
// branch: both lanes assemble the same encoding and share the permutations (keccakf_pair,
// 120 instead of 180 dependent VALU a round); one wave per block, the VGPR budget is free at
// this occupancy.
constexpr uint32_t SMALL_LEVEL = 32768;  // branches per level below which k_branch_small runs
constexpr uint32_t SMALL_BPB = 32;       // k_branch_small: branches per 64-lane block
__global__ void __launch_bounds__(64) k_branch_small(Topo T, uint64_t first, uint64_t cnt) {
  constexpr uint32_t WB = 64;
  __shared__ uint64_t slots[WB * LEAF_WORDS];
  __shared__ uint64_t crs[64 * WB];
  __shared__ uint16_t cms[16 * WB];
  const uint64_t t = (uint64_t)blockIdx.x * SMALL_BPB + (threadIdx.x >> 1);  // (a pair is inside or past cnt together)
  unsigned long long perms = 0, hashes = 0, inl = 0;
  if (t < cnt) {
    const uint32_t j = (uint32_t)(first + t), tid = threadIdx.x;
    const uint32_t k = T.br_k[j];
    const uint64_t cb = T.br_cbase[j];
    uint64_t r[64];
    uint32_t mm[16];
    if (T.cend) {  // leaf positions: the leaf children straight from their stashes (op_leaf_children)
      uint32_t ce[16];
#pragma unroll
      for (uint32_t c = 0; c < 16; ++c) {
        if (c < k) {
          mm[c] = T.cmeta[cb + c];
          ce[c] = T.cend[cb + c];
        }
      }
      const uint32_t d = T.br_depth[j];
      uint64_t pos = T.br_first[j];
#pragma unroll
      for (uint32_t c = 0; c < 16; ++c) {
        if (c < k) {
          const bool br = mm[c] & CM_BR;
          const uint64_t* src = br ? T.cref + 4 * (cb + c) : T.lf_eref + 4 * pos;
          const ulonglong2 a = ((const ulonglong2*)src)[0], b = ((const ulonglong2*)src)[1];
          r[4 * c] = a.x;
          r[4 * c + 1] = a.y;
          r[4 * c + 2] = b.x;
          r[4 * c + 3] = b.y;
          if (!br) mm[c] = (T.lf_inline ? T.lf_emeta[pos] : 32u) | (key_nibble(sorted_key(T, pos, d + 1), (int)d) << 8);
          pos = br ? ce[c] : pos + 1;
        }
      }
    } else {
#pragma unroll
      for (uint32_t c = 0; c < 16; ++c) {
        if (c < k) {
          const ulonglong2* p = (const ulonglong2*)(T.cref + 4 * (cb + c));
          const ulonglong2 a = p[0], b = p[1];
          r[4 * c] = a.x;
          r[4 * c + 1] = a.y;
          r[4 * c + 2] = b.x;
          r[4 * c + 3] = b.y;
          mm[c] = T.cmeta[cb + c];
        }
      }
    }
#pragma unroll
    for (uint32_t c = 0; c < 16; ++c) {
      if (c < k) {
        cms[c * WB + tid] = (uint16_t)mm[c];
#pragma unroll
        for (uint32_t q = 0; q < 4; ++q) crs[(4 * c + q) * WB + tid] = r[4 * c + q];
      }
    }
    uint32_t in1 = 0;
    perms = op_branch_stream_t<SRC_LDS, true>(T, j, slots + tid * LEAF_WORDS, 1, &in1, ChildSrc{cms + tid, crs + tid, WB});
    hashes = branch_hash_count(T, j, (uint32_t)perms);
    inl = in1;
    if (tid & 1) perms = hashes = inl = 0;  // (counted once per pair)
  }
  perms = wave_sum(perms);
  hashes = wave_sum(hashes);
  inl = wave_sum(inl);
  if (threadIdx.x == 0) {
    if (perms) atomicAdd(ctr_stat(T.ctr, CTR_PERMS, blockIdx.x), perms);
    if (hashes) atomicAdd(ctr_stat(T.ctr, CTR_HASHES, blockIdx.x), hashes);
    if (inl) atomicAdd(ctr_stat(T.ctr, CTR_INLINE, blockIdx.x), inl);
  }
}

// LDS ordering between lanes of ONE wave (the wave's LDS operations execute in
// order; the fences stop the compiler from moving them across): no block barrier
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// 16-lane inclusive prefix sum inside each DPP row (row_shr:1,2,4,8; lanes shifted in
// from outside the row read 0)
__device__ __forceinline__ uint32_t row16_scan(uint32_t x) {
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xF, 0xF, true);  // row_shr:1
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xF, 0xF, true);  // row_shr:2
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xF, 0xF, true);  // row_shr:4
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xF, 0xF, true);  // row_shr:8
  return x;
}

// The smallest levels (the top of a block commit's tries: 1, 16, 256, 4096 branches):
// 32 lanes per branch, two branches per wave.  Lane c < 16 loads child record c (one round
// trip for all 16), the item offsets are a DPP prefix sum over the group's first row, the
// items are XOR-placed (ds_xor) into the group's 0x80-prefilled encoding in LDS, and the
// permutation runs spread over the group (keccak_xlane.h): ~3x shorter than one thread's
// permutation, which at this occupancy is the level's latency.  Lane 0 of the group then
// keeps and publishes the reference as op_branch_stream does.
#ifndef KH_XL_LEVEL
#define KH_XL_LEVEL 8192
#endif
constexpr uint32_t XL_LEVEL = KH_XL_LEVEL;  // branches per level below which k_branch_xl runs
constexpr uint32_t XL_ENC_WORDS = 68;  // 4 windows: a branch of fixed-length keys is <= 532 B
__global__ void __launch_bounds__(64) k_branch_xl(Topo T, uint64_t first, uint64_t cnt) {
  __shared__ uint64_t enc[2][XL_ENC_WORDS];
  __shared__ uint64_t kb[2][64];
  const uint32_t g = threadIdx.x >> 5, sub = threadIdx.x & 31, gbase = threadIdx.x & 32u;
  const uint64_t t = (uint64_t)blockIdx.x * 2 + g;
  if (t >= cnt) return;  // the whole group (no cross-group operations below)
  const uint32_t j = (uint32_t)(first + t);
  uint64_t* E = enc[g];
  const uint32_t k = T.br_k[j];
  const uint64_t cb = T.br_cbase[j];
  const uint32_t ext = T.br_ext[j];
  const bool top = T.br_parent[j] == NONE;
  uint32_t len = 0, nib = 0;
  uint64_t r0 = 0, r1 = 0, r2 = 0, r3 = 0;
  uint32_t mc = 0, ce = 0;
  if (sub < k) {
    mc = T.cmeta[cb + sub];
    if (T.cend) ce = T.cend[cb + sub];
  }
  // leaf positions: a leaf child's stash is read where it lies -- child c sits right after the
  // last branch child b before it (at that branch's end, plus c - b - 1), or at the branch's
  // first key plus c (op_leaf_children, here one lane per child)
  const bool leafpos = T.cend && sub < k && !(mc & CM_BR);
  const uint32_t bm = (uint32_t)(__ballot(T.cend && sub < k && (mc & CM_BR)) >> gbase) & 0xFFFFu;
  const uint32_t below = sub < 16 ? bm & ((1u << sub) - 1) : 0;
  const int bl = below ? 31 - __builtin_clz(below) : -1;
  const uint32_t ceb = (uint32_t)__shfl((int)ce, (int)(gbase + (bl < 0 ? 0 : bl)));
  if (sub < k) {
    uint64_t pos = 0;
    if (leafpos) pos = bl < 0 ? (uint64_t)T.br_first[j] + sub : (uint64_t)ceb + (sub - (uint32_t)bl - 1);
    const ulonglong2* p = (const ulonglong2*)(leafpos ? T.lf_eref + 4 * pos : T.cref + 4 * (cb + sub));
    const ulonglong2 a = p[0], b = p[1];
    r0 = a.x, r1 = a.y, r2 = b.x, r3 = b.y;
    if (leafpos) {
      const uint32_t d = T.br_depth[j];
      mc = (T.lf_inline ? T.lf_emeta[pos] : 32u) | (key_nibble(sorted_key(T, pos, d + 1), (int)d) << 8);
    }
    len = mc & 0xFF;
    nib = (mc >> 8) & 0xF;
  }
  const uint32_t ilen = len == 32 ? 33 : len;
  const uint32_t incl = row16_scan(ilen ? ilen - 1 : 0);  // lanes 0..15 of the group: one DPP row
  const uint32_t sum = (uint32_t)__shfl((int)incl, (int)(gbase + 15));
  const uint32_t payload = 17 + sum;  // 16 - k empty slots + the terminator + sum of item lengths
  const uint32_t hh = rlp_hdr_len(payload), L = hh + payload;
  const bool hashit = L >= 32 || (top && ext == 0);
  const uint32_t nfull = L / 136;
  // 0x80 over the encoding's bytes, zero past them
  for (uint32_t w = sub; w < XL_ENC_WORDS; w += 32) {
    const uint32_t a = 8 * w, n80 = L > a ? (L - a < 8 ? L - a : 8) : 0;
    E[w] = low_bytes_mask(n80) & 0x8080808080808080ULL;
  }
  xl_sync();
  if (sub == 0) {  // the list header
    const uint64_t hdr = hh == 1 ? (0xC0 + payload)
                         : hh == 2 ? (0xF8 | ((uint64_t)payload << 8))
                                   : (0xF9 | ((uint64_t)(payload >> 8) << 8) | ((uint64_t)(payload & 0xFF) << 16));
    atomicXor((unsigned long long*)E, (unsigned long long)((hdr ^ 0x8080808080808080ULL) & low_bytes_mask(hh)));
  }
  if (ilen) {  // child sub's item (0xa0 + hash, or the embedded encoding) at its offset
    const uint32_t off = hh + nib + incl - (ilen - 1);
    uint64_t I[5];
    if (len == 32) {
      I[0] = 0xA0 | (r0 << 8);
      I[1] = (r0 >> 56) | (r1 << 8);
      I[2] = (r1 >> 56) | (r2 << 8);
      I[3] = (r2 >> 56) | (r3 << 8);
      I[4] = r3 >> 56;
    } else {
      I[0] = r0, I[1] = r1, I[2] = r2, I[3] = r3, I[4] = 0;
    }
    const uint32_t sh = off & 7, wfirst = off >> 3;
#pragma unroll
    for (uint32_t q = 0; q < 6; ++q) {
      const uint64_t cur = q < 5 ? I[q] : 0, prv = q ? I[q - 1] : 0;
      const uint64_t y = sh ? (cur << (8 * sh)) | (prv >> (64 - 8 * sh)) : cur;
      const uint32_t W = wfirst + q;
      const int32_t lo = (int32_t)off - 8 * (int32_t)W, hi = (int32_t)(off + ilen) - 8 * (int32_t)W;
      const uint32_t blo = lo > 0 ? (uint32_t)lo : 0, bhi = hi < 8 ? (hi > 0 ? (uint32_t)hi : 0) : 8;
      if (bhi <= blo) continue;
      const uint64_t m = low_bytes_mask(bhi) & ~low_bytes_mask(blo);
      atomicXor((unsigned long long*)(E + W), (unsigned long long)((y ^ 0x8080808080808080ULL) & m));
    }
  }
  xl_sync();
  // absorb + permute, spread over the group; the padding is added at absorb time so the
  // encoding stays intact in LDS (the inline reference of a short node)
  uint32_t lo = 0, hi = 0;
  if (hashit) {
    const XLane X = xlane_setup(sub);
    const uint32_t rem = L - 136 * nfull;
    for (uint32_t b = 0; b <= nfull; ++b) {
      if (sub < 17) {
        uint64_t w = E[17 * b + sub];
        if (b == nfull) {
          if ((rem >> 3) == sub) w ^= 0x01ULL << (8 * (rem & 7));
          if (sub == 16) w ^= 0x80ULL << 56;
        }
        lo ^= (uint32_t)w;
        hi ^= (uint32_t)(w >> 32);
      }
      keccakf_xlane(lo, hi, kb[g], X);
    }
  }
  uint64_t hb[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const uint32_t l = (uint32_t)__shfl((int)lo, (int)(gbase + q)), h = (uint32_t)__shfl((int)hi, (int)(gbase + q));
    hb[q] = hashit ? ((uint64_t)h << 32) | l : 0;
  }
  uint64_t bhead[4] = {0, 0, 0, 0};
  uint32_t ninl = hashit ? 0 : 1, perms = hashit ? nfull + 1 : 0;
  if (sub == 0) {
    T.br_len[j] = L;
    if (L < 32)
      for (int q = 0; q < 4; ++q) {
        const uint32_t base = 8u * (uint32_t)q;
        bhead[q] = base < L ? E[q] & low_bytes_mask(L - base < 8 ? L - base : 8) : 0;
      }
    branch_keep(T, j, L, hb, bhead);
  }
  if (ext == 0) {
    if (sub != 0) return;
    perms += branch_publish(T, j, L, hb, bhead, Slot{E, 1}, &ninl);
  } else {
    // the extension above it: lane 0 encodes it into the group's (zeroed) LDS words and the
    // permutation runs spread over the group too, as the branch's did (one lane's
    // permutation here was the level's longest step)
    PubCtx P;
    uint32_t XL = 0;
    xl_sync();  // (lane 0 has read the branch encoding's head)
    if (sub < 17) E[sub] = 0;
    xl_sync();
    if (sub == 0) {
      P = pub_ctx(T, j);
      pub_cend(T, j, P);
      XL = ext_encode(T, j, P, L, hb, bhead, Slot{E, 1});
    }
    XL = (uint32_t)__shfl((int)XL, (int)gbase);
    xl_sync();
    const bool xhash = XL >= 32 || top;
    uint32_t xlo = 0, xhi = 0;
    if (xhash) {
      const XLane X = xlane_setup(sub);
      if (sub < 17) {
        uint64_t w = E[sub];
        if ((XL >> 3) == sub) w ^= 0x01ULL << (8 * (XL & 7));
        if (sub == 16) w ^= 0x80ULL << 56;
        xlo = (uint32_t)w;
        xhi = (uint32_t)(w >> 32);
      }
      keccakf_xlane(xlo, xhi, kb[g], X);
    }
    uint64_t hx[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const uint32_t l = (uint32_t)__shfl((int)xlo, (int)(gbase + q)), h = (uint32_t)__shfl((int)xhi, (int)(gbase + q));
      hx[q] = xhash ? ((uint64_t)h << 32) | l : 0;
    }
    if (sub != 0) return;
    ext_finish(T, j, P, XL, hx, Slot{E, 1}, &ninl);
    perms += xhash ? 1 : 0;
  }
  atomicAdd(ctr_stat(T.ctr, CTR_PERMS, blockIdx.x), (unsigned long long)perms);
  atomicAdd(ctr_stat(T.ctr, CTR_HASHES, blockIdx.x), (unsigned long long)branch_hash_count(T, j, perms));
  if (ninl) atomicAdd(ctr_stat(T.ctr, CTR_INLINE, blockIdx.x), (unsigned long long)ninl);
}

// write-back emission: node q in [0, m + 2B): leaf q, or branch / extension of branch (q-m)/2.
// src/stride: the node's message words (stride m for one-block leaves, 1 otherwise).
__device__ __forceinline__ bool emit_node(const Topo& T, uint64_t B, uint64_t q, const uint64_t** src,
                                          uint64_t* stride, uint32_t* len, const uint64_t** hash) {
  *stride = 1;
  if (q < T.m) {
    uint32_t L = T.lf_len[q];
    bool top = T.lf_parent[q] == NONE;
    if (L <= LEAF_SHORT_MAX) {
      *src = T.lmsg + q;
      *stride = T.lstride;
    } else {
      *src = (const uint64_t*)(T.arena + T.lf_aoff[q]);
    }
    *len = L;
    *hash = T.lf_hash + 4 * q;
    return L >= 32 || top;
  }
  uint64_t j = (q - T.m) >> 1;
  bool top = T.br_parent[j] == NONE;
  bool has_ext = T.br_ext[j] != 0;
  bool is_ext = ((q - T.m) & 1) != 0;
  if (is_ext && !has_ext) return false;
  Slot sl = branch_slot(T, T.br_aoff[j], T.br_depth[j], is_ext);
  *src = sl.w;
  *stride = sl.stride;
  if (!is_ext) {
    uint32_t L = T.br_len[j];
    *len = L;
    *hash = T.br_hash + 4 * j;
    return L >= 32 || (top && !has_ext);
  }
  uint32_t L = T.ex_len[j];
  *len = L;
  *hash = T.ex_hash + 4 * j;
  return L >= 32 || top;
}

__global__ void __launch_bounds__(BS) k_emit_sizes(Topo T, uint64_t B, uint32_t* flag, uint64_t* bytes) {
  uint64_t q = (uint64_t)blockIdx.x * BS + threadIdx.x;
  if (q >= T.m + 2 * B) return;
  const uint64_t* src;
  uint64_t stride;
  uint32_t len;
  const uint64_t* h;
  bool e = emit_node(T, B, q, &src, &stride, &len, &h);
  if (T.emit_sel) e = e && T.emit_sel[q];
  flag[q] = e ? 1 : 0;
  bytes[q] = e ? len : 0;
}

__global__ void __launch_bounds__(BS) k_emit_copy(Topo T, uint64_t B, const uint32_t* pos, const uint64_t* boff,
                                                  uint8_t* out_hash, uint8_t* out_rlp, uint64_t* out_off) {
  uint64_t q = (uint64_t)blockIdx.x * BS + threadIdx.x;
  if (q >= T.m + 2 * B) return;
  const uint64_t* src;
  uint64_t stride;
  uint32_t len;
  const uint64_t* h;
  if (!emit_node(T, B, q, &src, &stride, &len, &h)) return;
  if (T.emit_sel && !T.emit_sel[q]) return;
  uint64_t p = pos[q];
  uint64_t* oh = (uint64_t*)(out_hash + 32 * p);
  for (int j = 0; j < 4; ++j) oh[j] = h[j];
  uint8_t* dst = out_rlp + boff[q];
  for (uint32_t b = 0; b < len; ++b) dst[b] = (uint8_t)(src[(b >> 3) * stride] >> (8 * (b & 7)));
  out_off[p] = boff[q];
}


// Copy L bytes between arbitrary byte addresses with a group of CG consecutive lanes
// (lane = 0..CG-1): word loads (load64u_n), whole-word stores where the destination is
// aligned, bytes at the unaligned ends.  The group's word stores are adjacent, so a
// wave writes 64/CG spans as contiguous runs instead of 64 scattered words.  Span
// gathers (resident merge, multi-GPU partition) are HBM-bound; one thread per span
// left them at <1 TB/s.
constexpr uint32_t CG = 8;
__device__ __forceinline__ void copy_bytes_group(uint8_t* dst, const uint8_t* src, uint64_t L, uint32_t lane) {
  uint64_t hb = (8 - ((uintptr_t)dst & 7)) & 7;
  if (hb > L) hb = L;
  if (lane < hb) dst[lane] = src[lane];
  const uint64_t nw = (L - hb) >> 3;
  for (uint64_t w = lane; w < nw; w += CG)
    *(uint64_t*)(dst + hb + 8 * w) = load64u_n(src + hb + 8 * w, 8);
  const uint64_t t0 = hb + 8 * nw;
  if (t0 + lane < L) dst[t0 + lane] = src[t0 + lane];
}

// ---- multi-GPU routing: stable partition of records by top-nibble owner
__device__ __forceinline__ uint32_t nibble_owner(uint64_t w0, uint32_t nparts) {
  return (((uint32_t)(w0 & 0xFF) >> 4) * nparts) >> 4;
}
// Stable partition in source order, three passes over tiles of PT_TILE consecutive
// records: k_part_count (records per owner per tile), an exclusive scan of that
// owner-major table (= the first destination of every (owner, tile)), k_part_place
// (each record's destination: the tile base + its rank among the tile's earlier records
// of the same owner; keys and lengths written there), a scan of the placed lengths
// (value byte offsets), then k_part_vcopy copies the value spans in source order
// (coalesced reads; each record's bytes go to one contiguous destination run).
constexpr uint32_t PT_R = 8;
constexpr uint64_t PT_TILE = (uint64_t)BS * PT_R;
constexpr uint32_t PT_WAVES = BS / 64;
// lanes of this wave with the same owner (owners < 32; invalid lanes excluded)
__device__ __forceinline__ uint64_t owner_match(bool ok, uint32_t o) {
  uint64_t mask = __ballot(ok);
  for (int b = 0; b < 5; ++b) {
    const bool bit = (o >> b) & 1;
    const uint64_t m = __ballot(ok && bit);
    mask &= bit ? m : ~m;
  }
  return mask;
}
__global__ void __launch_bounds__(BS) k_part_count(const uint64_t* K, uint64_t n, uint32_t nparts, uint32_t ntile,
                                                   uint32_t* hist) {
  __shared__ uint32_t c[16];
  if (threadIdx.x < 16) c[threadIdx.x] = 0;
  __syncthreads();
  const uint64_t t0 = (uint64_t)blockIdx.x * PT_TILE;
  for (uint32_t r = 0; r < PT_R; ++r) {
    const uint64_t i = t0 + r * BS + threadIdx.x;
    const bool ok = i < n;
    const uint32_t o = ok ? nibble_owner(K[4 * i], nparts) : 0;
    const uint64_t mask = owner_match(ok, o);
    if (ok && (mask & lanemask_lt()) == 0) atomicAdd(&c[o], (uint32_t)__popcll(mask));  // one add per group
  }
  __syncthreads();
  if (threadIdx.x < nparts) hist[(uint64_t)threadIdx.x * ntile + blockIdx.x] = c[threadIdx.x];
}
// the owners' record counts (the scanned tile table) and value bytes (the sum of the tiles'
// byte sums, k_part_place's hbytes): block p for owner p
__global__ void __launch_bounds__(BS) k_part_bounds_t(const uint32_t* base, const unsigned long long* hbytes,
                                                      uint32_t ntile, uint64_t n, uint32_t nparts,
                                                      unsigned long long* cnt, unsigned long long* bytes) {
  __shared__ unsigned long long part[PT_WAVES];
  const uint32_t p = blockIdx.x;
  unsigned long long v = 0;
  for (uint32_t t = threadIdx.x; t < ntile; t += BS) v += hbytes[(uint64_t)p * ntile + t];
  v = wave_sum(v);
  if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = v;
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned long long tot = 0;
    for (uint32_t w = 0; w < PT_WAVES; ++w) tot += part[w];
    bytes[p] = tot;
    const uint64_t a = base[(uint64_t)p * ntile];
    const uint64_t b = p + 1 < nparts ? base[(uint64_t)(p + 1) * ntile] : n;
    cnt[p] = b - a;
  }
}
// Key hashing for kh_dev_hash_partition_ev: each key's owner also goes out as one byte, so
// the count pass (k_part_count_o) reads 1 byte per record instead of the keys' lines
template <bool SHORT>
__device__ __forceinline__ void hash_keys_owner(const uint8_t* keys, uint32_t klen, uint64_t n, uint64_t* out,
                                                uint32_t nparts, uint8_t* owner) {
  const uint64_t i = (uint64_t)blockIdx.x * BS + threadIdx.x;
  if (i >= n) return;
  uint64_t h[4];
  if (SHORT)
    kec256_short(keys + i * klen, klen, h);
  else
    kec256_msg<false>(keys + i * klen, klen, h);
  for (int j = 0; j < 4; ++j) out[4 * i + j] = h[j];
  owner[i] = (uint8_t)nibble_owner(h[0], nparts);
}
__global__ void __launch_bounds__(BS) __attribute__((amdgpu_waves_per_eu(7)))
k_hash_keys_owner_s(const uint8_t* keys, uint32_t klen, uint64_t n, uint64_t* out, uint32_t nparts, uint8_t* owner) {
  hash_keys_owner<true>(keys, klen, n, out, nparts, owner);
}
__global__ void __launch_bounds__(BS) k_hash_keys_owner_l(const uint8_t* keys, uint32_t klen, uint64_t n,
                                                          uint64_t* out, uint32_t nparts, uint8_t* owner) {
  hash_keys_owner<false>(keys, klen, n, out, nparts, owner);
}
// k_part_count from the owner bytes: PT_R consecutive records per thread (one 8-byte load),
// counted per owner in registers, one wave sum and LDS add per owner
__global__ void __launch_bounds__(BS) k_part_count_o(const uint8_t* owner, uint64_t n, uint32_t nparts, uint32_t ntile,
                                                     uint32_t* hist) {
  static_assert(PT_R == 8, "one 8-byte load per thread");
  __shared__ uint32_t c[16];
  if (threadIdx.x < 16) c[threadIdx.x] = 0;
  __syncthreads();
  const uint64_t i0 = (uint64_t)blockIdx.x * PT_TILE + (uint64_t)threadIdx.x * PT_R;
  uint64_t w = 0;
  if (i0 + PT_R <= n) {
    w = *(const uint64_t*)(owner + i0);
  } else {
    for (uint32_t r = 0; r < PT_R; ++r)
      if (i0 + r < n) w |= (uint64_t)owner[i0 + r] << (8 * r);
  }
  const uint32_t valid = i0 >= n ? 0u : (uint32_t)min<uint64_t>(PT_R, n - i0);
  uint32_t acc[16];
#pragma unroll
  for (uint32_t q = 0; q < 16; ++q) acc[q] = 0;
#pragma unroll
  for (uint32_t r = 0; r < PT_R; ++r) {
    const uint32_t o = (uint32_t)(w >> (8 * r)) & 0xFF;
#pragma unroll
    for (uint32_t q = 0; q < 16; ++q) acc[q] += (r < valid && o == q) ? 1u : 0u;
  }
#pragma unroll
  for (uint32_t q = 0; q < 16; ++q) {
    if (q < nparts) {
      const uint32_t v = wave_sum(acc[q]);
      if ((threadIdx.x & 63) == 0 && v) atomicAdd(&c[q], v);
    }
  }
  __syncthreads();
  if (threadIdx.x < nparts) hist[(uint64_t)threadIdx.x * ntile + blockIdx.x] = c[threadIdx.x];
}
// V16: keys in and out 16-byte aligned -- each key moved as two 16-byte loads issued before
// the round's ranking and two 16-byte stores (8-byte words otherwise)
template <bool V16>
__global__ void __launch_bounds__(BS) k_part_place(const uint64_t* K, const uint64_t* voff, uint64_t n,
                                                   uint32_t nparts, uint32_t ntile, const uint32_t* base,
                                                   uint64_t* okeys, uint64_t* olen, uint32_t* pos,
                                                   unsigned long long* hbytes) {
  // (hbytes: the tile's value bytes per owner -- the owners' byte totals without a scan of
  // the placed lengths, which then runs after the counts are back)
  __shared__ uint32_t run[16];
  __shared__ uint32_t wc[PT_WAVES][16];
  __shared__ unsigned long long cb[16];
  const uint32_t wv = threadIdx.x >> 6;
  if (threadIdx.x < 16) run[threadIdx.x] = threadIdx.x < nparts ? base[(uint64_t)threadIdx.x * ntile + blockIdx.x] : 0;
  if (threadIdx.x < 16) cb[threadIdx.x] = 0;
  uint64_t acc[16];
#pragma unroll
  for (uint32_t q = 0; q < 16; ++q) acc[q] = 0;
  const uint64_t t0 = (uint64_t)blockIdx.x * PT_TILE;
  for (uint32_t r = 0; r < PT_R; ++r) {
    if (threadIdx.x < PT_WAVES * 16) wc[threadIdx.x >> 4][threadIdx.x & 15] = 0;
    __syncthreads();
    const uint64_t i = t0 + r * BS + threadIdx.x;
    const bool ok = i < n;
    ulonglong2 k0 = make_ulonglong2(0, 0), k1 = make_ulonglong2(0, 0);
    uint64_t len = 0;
    if (ok) {
      if (V16) {
        k0 = ((const ulonglong2*)K)[2 * i];
        k1 = ((const ulonglong2*)K)[2 * i + 1];
      } else {
        k0 = make_ulonglong2(K[4 * i], K[4 * i + 1]);
        k1 = make_ulonglong2(K[4 * i + 2], K[4 * i + 3]);
      }
      len = voff[i + 1] - voff[i];
    }
    const uint32_t o = ok ? nibble_owner(k0.x, nparts) : 0;
    const uint64_t mask = owner_match(ok, o);
    const uint32_t rk = (uint32_t)__popcll(mask & lanemask_lt());
    if (ok && rk == 0) wc[wv][o] = (uint32_t)__popcll(mask);
    __syncthreads();
    if (ok) {
      uint32_t d = run[o] + rk;
      for (uint32_t w = 0; w < wv; ++w) d += wc[w][o];
      pos[i] = d;
      if (V16) {
        ((ulonglong2*)okeys)[2 * (uint64_t)d] = k0;
        ((ulonglong2*)okeys)[2 * (uint64_t)d + 1] = k1;
      } else {
        okeys[4 * (uint64_t)d] = k0.x;
        okeys[4 * (uint64_t)d + 1] = k0.y;
        okeys[4 * (uint64_t)d + 2] = k1.x;
        okeys[4 * (uint64_t)d + 3] = k1.y;
      }
      olen[d] = len;
    }
#pragma unroll
    for (uint32_t q = 0; q < 16; ++q) acc[q] += o == q ? len : 0ull;
    __syncthreads();
    if (threadIdx.x < nparts) {
      uint32_t t = 0;
      for (uint32_t w = 0; w < PT_WAVES; ++w) t += wc[w][threadIdx.x];
      run[threadIdx.x] += t;
    }
    __syncthreads();
  }
#pragma unroll
  for (uint32_t q = 0; q < 16; ++q) {
    if (q < nparts) {
      const unsigned long long v = wave_sum((unsigned long long)acc[q]);
      if ((threadIdx.x & 63) == 0 && v) atomicAdd(&cb[q], v);
    }
  }
  __syncthreads();
  if (threadIdx.x < nparts) hbytes[(uint64_t)threadIdx.x * ntile + blockIdx.x] = cb[threadIdx.x];
}
// Value spans to their placed offsets, in source order: one CG-lane group per record
// (consecutive groups read consecutive source bytes)
__global__ void __launch_bounds__(BS) k_part_vcopy(const uint8_t* vals, const uint64_t* voff, const uint32_t* pos,
                                                   const uint64_t* ooff, uint64_t n, uint8_t* ovals) {
  const uint64_t i = ((uint64_t)blockIdx.x * BS + threadIdx.x) / CG;
  const uint32_t lane = threadIdx.x % CG;
  if (i >= n) return;
  const uint64_t o = voff[i];
  copy_bytes_group(ovals + ooff[pos[i]], vals + o, voff[i + 1] - o, lane);
}
__global__ void __launch_bounds__(BS) k_synth_len(uint32_t cfg, uint64_t first, uint64_t n, uint64_t* voff) {
  uint64_t i = (uint64_t)blockIdx.x * BS + threadIdx.x;
  if (i > n) return;
  voff[i] = (i < n) ? synth_body_len(synth_acct(cfg, first + i)) : 0;
}

__global__ void __launch_bounds__(BS) k_synth_write(uint32_t cfg, uint64_t first, uint64_t n, const uint64_t* voff,
                                                    uint8_t* addr, uint8_t* vals) {
  uint64_t i = (uint64_t)blockIdx.x * BS + threadIdx.x;
  if (i >= n) return;
  SynthAcct a = synth_acct(cfg, first + i);
  synth_addr_write(a, addr + 20 * i);
  synth_body_write(a, first + i, vals + voff[i]);
}

// ---------------------------------------------------------------------------
// device workspace
// ---------------------------------------------------------------------------
// selects device d (d >= 0) for the guard's scope, restoring the caller's device after
struct DevScope {
  int prev = -1;
  explicit DevScope(int d) {
    int cur = -1;
    if (d >= 0 && hipGetDevice(&cur) == hipSuccess && cur != d && hipSetDevice(d) == hipSuccess) prev = cur;
  }
  ~DevScope() {
    if (prev >= 0) (void)hipSetDevice(prev);
  }
  DevScope(const DevScope&) = delete;
  DevScope& operator=(const DevScope&) = delete;
};

// A device buffer that remembers the GPU it lives on: growth drains and frees on THAT
// device, and allocates on `on` (or on the current device when on < 0).
struct DevBuf {
  void* p = nullptr;
  size_t cap = 0;
  int dev = -1;
  DevBuf() = default;
  DevBuf(const DevBuf&) = delete;
  DevBuf& operator=(const DevBuf&) = delete;
  ~DevBuf() { release(); }  // a throw between ensure() and release() does not leak HBM
  void ensure(size_t bytes, int on = -1) {
    if (on < 0) {
      if (hipGetDevice(&on) != hipSuccess) on = 0;
    }
    if (bytes <= cap && dev == on) return;
    if (p) {
      // work still reading the old buffer may be in flight (kh_dev_partition_ev returns before
      // its value copy ends): drain its device before the buffer goes (growth is rare)
      DevScope ds(dev);
      HIPCHK(hipDeviceSynchronize());
      HIPCHK(hipFree(p));
    }
    p = nullptr;
    cap = 0;
    size_t want = bytes + bytes / 8 + 4096;
    DevScope ds(on);
    HIPCHK(hipMalloc(&p, want));
    cap = want;
    dev = on;
  }
  void release() {
    if (p) {
      DevScope ds(dev);
      (void)hipFree(p);
    }
    p = nullptr;
    cap = 0;
    dev = -1;
  }
};

// bump carving inside one DevBuf
struct Carver {
  char* base;
  size_t off = 0;
  size_t cap;
  template <typename T>
  T* take(size_t count) {
    off = (off + 255) & ~(size_t)255;
    T* r = (T*)(base + off);
    off += count * sizeof(T) + 16;  // +16: slack for 8-byte word over-reads
    if (off > cap) throw KhError{KH_EINTERNAL, "workspace carve overflow"};
    return r;
  }
};
static size_t carve_size(const std::vector<size_t>& items) {
  size_t s = 0;
  for (size_t b : items) s = ((s + 255) & ~(size_t)255) + b + 16;
  return s + 256;
}

struct BuildInfo {  // the last build's sizes, for build_stats
  uint64_t n = 0, m = 0, B = 0, key_perms = 0, arena = 0;
  uint32_t levels = 0;
  bool full_sort = false, early = false, stage_ev = true;
};
// A host thread kept for a context (kh_block_commit's storage phase): post() hands it one job,
// join() waits for the job; no thread is started per call.
struct Worker {
  std::thread th;
  std::mutex mu;
  std::condition_variable cv;
  std::function<void()> job;
  bool has_job = false, stop = false;
  void post(std::function<void()> f) {
    std::unique_lock<std::mutex> lk(mu);
    if (!th.joinable()) th = std::thread([this] { loop(); });
    job = std::move(f);
    has_job = true;
    cv.notify_all();
  }
  void join() {
    std::unique_lock<std::mutex> lk(mu);
    cv.wait(lk, [this] { return !has_job; });
  }
  void loop() {
    std::unique_lock<std::mutex> lk(mu);
    for (;;) {
      cv.wait(lk, [this] { return has_job || stop; });
      if (stop) return;
      std::function<void()> f = std::move(job);
      lk.unlock();
      f();  // (the job catches its own exceptions)
      lk.lock();
      has_job = false;
      cv.notify_all();
    }
  }
  ~Worker() {
    {
      std::lock_guard<std::mutex> lk(mu);
      stop = true;
    }
    cv.notify_all();
    if (th.joinable()) th.join();
  }
};

// Host memcpy into pinned staging on COPY_THREADS host threads (the caller and COPY_THREADS - 1
// kept workers): a single thread copies pageable -> pinned at ~22 GB/s on the box, 4 threads at
// ~80, 8 at ~113, against ~57 GB/s of PCIe (profiles/r8a_h2d_probe.jsonl).  One job at a time,
// split into one part per thread, so a worker never mixes parts of two jobs.
constexpr int COPY_THREADS = 8;
class CopyPool {
  std::vector<std::thread> th_;
  std::mutex job_mu_, mu_;
  std::condition_variable cv_, done_;
  uint8_t* dst_ = nullptr;
  const uint8_t* src_ = nullptr;
  size_t bytes_ = 0, part_ = 0;
  uint64_t gen_ = 0;
  int left_ = 0;
  bool stop_ = false;
  void part(int w) {
    const size_t a = part_ * (size_t)w;
    if (a < bytes_) memcpy(dst_ + a, src_ + a, std::min(part_, bytes_ - a));
  }
  void loop(int w) {
    uint64_t seen = 0;
    std::unique_lock<std::mutex> lk(mu_);
    for (;;) {
      cv_.wait(lk, [&] { return stop_ || gen_ != seen; });
      if (stop_) return;
      seen = gen_;
      lk.unlock();
      part(w);
      lk.lock();
      if (--left_ == 0) done_.notify_all();
    }
  }

 public:
  void copy(void* dst, const void* src, size_t bytes) {
    if (bytes < (8u << 20)) {  // (a small copy is not worth the hand-off)
      memcpy(dst, src, bytes);
      return;
    }
    std::lock_guard<std::mutex> jl(job_mu_);
    std::unique_lock<std::mutex> lk(mu_);
    for (int w = (int)th_.size() + 1; w < COPY_THREADS; ++w) th_.emplace_back([this, w] { loop(w); });
    dst_ = (uint8_t*)dst;
    src_ = (const uint8_t*)src;
    bytes_ = bytes;
    part_ = ((bytes + COPY_THREADS - 1) / COPY_THREADS + 4095) & ~(size_t)4095;
    left_ = COPY_THREADS - 1;
    ++gen_;
    cv_.notify_all();
    lk.unlock();
    part(0);
    lk.lock();
    done_.wait(lk, [&] { return left_ == 0; });
  }
  ~CopyPool() {
    {
      std::lock_guard<std::mutex> lk(mu_);
      stop_ = true;
    }
    cv_.notify_all();
    for (auto& t : th_) t.join();
  }
};
static CopyPool g_copy_pool;
constexpr int RING_SLOTS = 4;
constexpr size_t RING_CHUNK = 64u << 20;  // 64 MB chunks: 56 GB/s end to end in the probe (32-128 MB alike)
struct kh_ctx {
  int dev = 0;
  int n_cu = 256;  // compute units of the device
  hipStream_t own = nullptr;
  hipStream_t st = nullptr;
  hipStream_t st2 = nullptr;  // leaf hashing, concurrent with the branch topology
  // every entry point that uses the context holds it (recursive: a *_host entry point locks,
  // then calls its device variant, which locks again); a resident handle's calls lock the
  // context the handle was opened on (kh_trie::home)
  std::recursive_mutex mu;
  DevBuf ws_list;  // element builds: the list of leaves to hash (k_leaf_prep -> k_leaf_hash_list)
  DevBuf ws_inject;                    // kh_block_commit: the injection's error word
  unsigned long long inject_tok = 0;   //   and the token the last call writes there on error
  DevBuf ws_arena;  // the build's long leaves (sized once the leaves are hashed)
  DevBuf ws1, ws2, ws3, in_keys, in_vals, in_voff, in_seg, in_kn, in_aux, in_block, out_emit, emit_dev;
  hipEvent_t ev[11] = {};  // [0..5] build stages (st), [6] / [7] forest commit marks, [8] boundaries
                          // ready (st), [9] / [10] leaf kernel start / end (st2)
  unsigned long long* h_pinned = nullptr;  // small pinned staging for syncs
  uint8_t* h_res = nullptr;                // pinned staging of the per-result outputs (grown; a pageable
  size_t h_res_cap = 0;                    // copy of 100k roots cost 20-30 ms of page pinning per build)
  // kh_block_commit: the second context its storage phase runs on, beside the account phase on
  // this one, and the event of the storage roots' injection into the account bodies
  kh_ctx* bsub = nullptr;
  hipEvent_t bev = nullptr;
  std::unique_ptr<Worker> bworker;
  // plain builds on the 32-bit-prefix path do not wait for the tie kernel's flags (SortIO::
  // speculate); a build whose flags were set (repeated keys, a long run) is redone without, and
  // the next spec_off builds do not speculate
  uint32_t spec_off = 0;
  // last build (for emission)
  Topo T{};
  uint64_t last_B = 0;
  uint64_t last_nres = 0;
  BuildInfo binfo;
  // host-input staging (HostStage): a copy stream, a ring of pinned chunks with the event of
  // each chunk's last DMA, the events the stager records (key parts, keys + offsets, values) and
  // the thread that streams the inputs behind the build (created on first use)
  hipStream_t cs = nullptr;
  uint8_t* ring = nullptr;
  hipEvent_t ring_ev[RING_SLOTS] = {};
  bool ring_busy[RING_SLOTS] = {};
  uint32_t ring_next = 0;
  std::vector<hipEvent_t> part_ev;
  std::unique_ptr<Worker> hworker;
  // small host inputs (a commit's ops: HostPack): packed into one pinned buffer, one DMA into
  // in_block; pack_ev marks that DMA (the next pack waits for it before reusing the buffer)
  uint8_t* h_pack = nullptr;
  size_t h_pack_cap = 0;
  hipEvent_t pack_ev = nullptr;
  bool pack_busy = false;
  bool pack_for_block = false;  // kh_block_commit_host -> kh_block_commit: its phases wait for pack_ev
};

// Host inputs (keys, value offsets, values of kh_trie_root / kh_trie_root_nodes /
// kh_trie_open_host) streamed to HBM behind the build instead of before it: the library's
// worker thread copies them through a ring of pinned 64-MB chunks (g_copy_pool's threads fill a
// chunk, one DMA on c->cs sends it) in the order the build needs them -- the keys in parts
// (an event each: key hashing starts on the first part while the others are in flight), then
// the value offsets (rebased on the device, not in a host copy), then the values.  The build
// waits for an event only where it first reads those bytes (the keys' parts at hashing, the
// values at the leaves), and the host waits for the worker to have RECORDED an event before
// enqueueing a wait on it (a wait on an unrecorded event would be a no-op).  Round 5 staged
// everything serially before the build: pageable copies plus an 800-MB host rebase of the
// offsets, 420 ms for 100M accounts (BENCH_r05 drop_in_host_path).
struct HostStage {
  kh_ctx* c;
  std::mutex mu;
  std::condition_variable cv;
  uint32_t recorded = 0;  // events recorded: key parts [0, nkp), then keys + offsets (nkp), values (nkp + 1)
  bool failed = false;
  int code = KH_OK;
  std::string msg;
  uint32_t nkp = 0;
  std::vector<uint64_t> kend;  // key part p covers inputs [kend[p-1], kend[p])
  bool posted = false;
  explicit HostStage(kh_ctx* cc) : c(cc) {}
  HostStage(const HostStage&) = delete;
  hipEvent_t ev(uint32_t p) const { return c->part_ev[p]; }
  // host: block until event p is recorded (throws the stager's error)
  void wait(uint32_t p) {
    std::unique_lock<std::mutex> lk(mu);
    cv.wait(lk, [&] { return recorded > p || failed; });
    if (recorded <= p) throw KhError{code, msg};
  }
  // host + stream: st waits for event p
  void stream_wait(hipStream_t st, uint32_t p) {
    wait(p);
    HIPCHK(hipStreamWaitEvent(st, ev(p), 0));
  }
  void publish() {
    std::lock_guard<std::mutex> lk(mu);
    ++recorded;
    cv.notify_all();
  }
  void join() {
    if (posted) c->hworker->join();
    posted = false;
  }
  ~HostStage() { join(); }  // the stager must be done with the staging buffers before the call returns
};

// ---------------------------------------------------------------------------
// the build
// ---------------------------------------------------------------------------
struct BuildArgs {
  const uint8_t* keys;
  uint32_t klen;
  const uint8_t* vals;
  const uint64_t* voff;  // [n+1] offsets, or with vlen: [n] offsets of spans anywhere in vals
  uint64_t n;
  const uint32_t* seg;  // nullable
  uint64_t nseg;
  uint32_t depth0;
  uint32_t flags;
  bool emit;
  const uint32_t* vlen = nullptr;  // per-input value lengths (element builds: spans in a value heap)
  const uint8_t* kn = nullptr;     // variable-length keys (zero-padded to 32 B): nibble counts (list tries)
  struct ElemArgs* el = nullptr;   // element build of a resident forest commit (forest.h; nullable)
  hipEvent_t vals_ready = nullptr; // the values / offsets land later (multi-GPU exchange): wait before reading them
  bool dev_results = false;        // results and counters stay on the device (no host sync at the end)
  bool no_spec = false;            // no speculative sort (SortIO::speculate): the retry of one that failed
  std::function<void()> before_leaves;  // element builds: called (host) right before the leaves are encoded
  std::function<bool()> late_ready;     // ... late values (ElemArgs::late) already on the device: one leaf pass
  HostStage* hs = nullptr;  // host inputs still streaming in (keys in parts, values last; vals_ready unset)
};
// element build (forest.h): inputs are leaves and subtree elements; the capped reference
// of every element node, branch and extension is kept for the forest's records
struct ElemArgs {
  const uint8_t* db;     // [n] EL_LEAF or subtree branch depth (input order)
  const uint64_t* bref;  // [n*4]
  const uint8_t* brl;    // [n]
  const uint8_t* oldd;   // [n] previous anchor depth (EL_NEW: none)
  const uint64_t* cref;  // [n*4] previous capped reference
  const uint8_t* crl;    // [n]
  // [n] nullable: the element's value arrives late (kh_block_commit: an account body that gets
  // its storage root): the other leaves are encoded and hashed before before_leaves
  const uint8_t* late = nullptr;
  DevBuf* out;           // sorted el_db / el_bref / el_brl and lf_ref / lf_rlen (sized by m)
  DevBuf* outb;          // br_ref / br_rlen, ex_ref / ex_rlen (sized by B)
};
struct BuildOut {
  std::vector<uint64_t> res_hash;  // nres*4
  std::vector<uint32_t> res_len;
  std::vector<uint64_t> res_inl;
};

constexpr uint32_t CK_KEY_BITS = 12;  // segmented ck path: fewest key bits left in the 32-bit sort word
static uint32_t bits_for(uint64_t nseg) {
  uint32_t b = 0;
  while (b < 64 && (1ULL << b) < nseg) ++b;
  return b;
}

// the context's pinned result staging, grown to at least `bytes` (the device is drained
// first: an earlier copy into the old buffer may still be in flight)
static uint8_t* pinned_stage(kh_ctx* c, size_t bytes) {
  if (bytes > c->h_res_cap) {
    HIPCHK(hipStreamSynchronize(c->st));
    if (c->h_res) HIPCHK(hipHostFree(c->h_res));
    c->h_res = nullptr;
    c->h_res_cap = 0;
    HIPCHK(hipHostMalloc((void**)&c->h_res, bytes + bytes / 4 + 4096, hipHostMallocDefault));
    c->h_res_cap = bytes + bytes / 4 + 4096;
  }
  return c->h_res;
}

// a speculative sort (SortIO::speculate) met repeated keys or a long run: the build is redone
struct SpecRetry {};

static float ev_ms(hipEvent_t a, hipEvent_t b) {
  float ms = 0;
  if (hipEventElapsedTime(&ms, a, b) != hipSuccess) return 0;
  return ms;
}

// Sort n 32-byte keys (with optional segment ids) and drop duplicates, keeping the
// last of equal keys.  Outputs the sorted keys, the input index of each and m.
struct SortIO {
  const uint64_t* K32;
  const uint32_t* seg;
  uint32_t sb;
  uint64_t n;
  uint64_t *ck0, *ck1;
  uint32_t *idx0, *idx1;
  uint64_t* skey;
  uint32_t* sseg;
  void* rs_scratch;
  void* scan_scratch;
  unsigned long long* ctr;
  const uint8_t* kn;  // variable-length keys: nibble counts (input order; nullable)
  bool ck_ready = false;  // ck_path: ck0/idx0 already hold the 32-bit sort keys (k_hash_keys_ck)
  bool ck_path = false;   // unsegmented plain build: sort (32-bit prefix, idx) only, never gather the keys
  bool ck_made = false;   // composite path: ck0 / idx0 and the radix header already made (k_f_keys_ck)
  // 64-bit composite path: the radix range is bits [rs_lo, 64) -- 40 (the leading 24 bits) where
  // keys are few per segment, the tie kernel then orders the runs of equal leading 24 bits
  int rs_lo = 32;
  // ck path: the words are sorted on their bits from tsh up (8: hashed keys, few enough that
  // runs of equal top-24 bits stay rare; the tie kernel orders them)
  uint32_t tsh = 0;
  // a device word copied to the host with the first sync's flags (c->h_pinned[1]): the
  // caller's check of earlier stream work, read without a sync of its own (nullable)
  const unsigned long long* chk = nullptr;
  // ck_path: no sync for the tie kernel's flags: the sort proceeds as if no key repeats and no
  // run is too long (hashed keys: the rule); the caller reads the flags at its next sync
  // (CTR_TIE) and redoes the build without speculating if either is set
  bool speculate = false;
  // out
  uint8_t* u = nullptr;  // ck_path: boundary values, written for the tie runs' inner boundaries
  uint32_t depth0 = 0;
  const uint32_t* sck = nullptr;  // ck_path: the sorted 32-bit key prefixes (skey not gathered)
  bool ties_u = false;            // u holds the tie runs' boundaries (k_lcp skips them)
  bool all_u = false;             // u holds every boundary (k_lcp only clears a too-long run's)
  uint64_t m;
  uint32_t* sidx;
  bool fallback;
};
static void sort_dedup(kh_ctx* c, SortIO& S) {
  hipStream_t st = c->st;
  if (S.chk && (S.ck_path || S.speculate)) throw KhError{KH_EINTERNAL, "sort: a check word on a speculative sort"};
  const uint64_t n = S.n;
  const uint64_t* K32 = S.K32;
  const uint32_t* seg = S.seg;
  const uint32_t sb = S.sb;
  const bool segmented = seg != nullptr;
  uint64_t *ck0 = S.ck0, *ck1 = S.ck1;
  uint32_t *idx0 = S.idx0, *idx1 = S.idx1;
  uint64_t* skey = S.skey;
  uint32_t* sseg = S.sseg;
  void* rs_scratch = S.rs_scratch;
  void* scan_scratch = S.scan_scratch;
  struct {
    unsigned long long* ctr;
  } T{S.ctr};
  // ---- 2. sort: LSD radix on the top 32 bits of the composite (segment | key) prefix,
  // then fix the rare runs of equal prefixes locally (k_tie_fix); a full 256-bit sort
  // only if a run is longer than TIE_RUN_MAX (adversarial keys)
  uint64_t* cks = nullptr;
  uint32_t* idxs = nullptr;
  bool long_run = false;  // the plain path met a run longer than TIE_RUN_MAX: full sort
  if (S.ck_path) {  // 32-bit prefixes: 8 bytes a pair per radix pass
    uint32_t* c0 = (uint32_t*)ck0;
    uint32_t* c1 = (uint32_t*)ck1;
    if (!S.ck_ready) {
      hipLaunchKernelGGL(k_make_ck32, GRID(n, BS), dim3(BS), 0, st, (const uint64_t*)K32, n, c0, idx0, seg, sb);
      LAUNCH_CHECK();
    }
    const bool flip = radix_sort_pairs<uint32_t>(c0, idx0, c1, idx1, n, S.tsh, 32, rs_scratch, st);
    uint32_t* c32 = flip ? c1 : c0;
    idxs = flip ? idx1 : idx0;
    const bool full_u = S.u && !segmented;
    hipLaunchKernelGGL(k_tie_fix_ck_blk, GRID(n, TF_ITEMS * BS), dim3(BS), 0, st, c32, idxs, n,
                       (const uint64_t*)K32, T.ctr + CTR_TIE, S.u, S.depth0, full_u, S.tsh);
    LAUNCH_CHECK();
    uint64_t tf = 0;
    if (!S.speculate) {
      HIPCHK(hipMemcpyAsync(c->h_pinned, T.ctr + CTR_TIE, 8, hipMemcpyDeviceToHost, st));
      HIPCHK(hipStreamSynchronize(st));
      tf = c->h_pinned[0];
    }
    long_run = tf & 1;
    if (!long_run) {
      uint64_t m = n;
      uint32_t* ock = c32;
      uint32_t* oidx = idxs;
      if (tf & 2) {  // keep the last of equal keys
        uint32_t* keep = c32 == c0 ? c1 : c0;
        uint32_t* keep_pos = idxs == idx0 ? idx1 : idx0;
        hipLaunchKernelGGL(k_dup_ck, GRID(n, BS), dim3(BS), 0, st, (const uint32_t*)c32, (const uint32_t*)idxs,
                           (const uint64_t*)K32, n, keep);
        LAUNCH_CHECK();
        uint32_t* mtot = (uint32_t*)(T.ctr + CTR_M);
        scan_exclusive<uint32_t>(keep, keep_pos, n, mtot, scan_scratch, st);
        HIPCHK(hipMemcpyAsync(c->h_pinned, mtot, 4, hipMemcpyDeviceToHost, st));
        HIPCHK(hipStreamSynchronize(st));
        m = (uint32_t)c->h_pinned[0];
        c->ws3.ensure(carve_size({n * 4, n * 4}));
        Carver c3{(char*)c->ws3.p, 0, c->ws3.cap};
        ock = c3.take<uint32_t>(n);
        oidx = c3.take<uint32_t>(n);
        hipLaunchKernelGGL(k_compact_ck, GRID(n, BS), dim3(BS), 0, st, (const uint32_t*)c32, (const uint32_t*)idxs,
                           (const uint32_t*)keep_pos, (const uint32_t*)keep, n, ock, oidx);
        LAUNCH_CHECK();
      }
      if (segmented) {  // the sorted segment ids (result_index, segment breaks) from the words
        hipLaunchKernelGGL(k_sseg_from_ck, GRID(m, BS), dim3(BS), 0, st, (const uint32_t*)ock, m, sb, sseg);
        LAUNCH_CHECK();
      }
      S.m = m;
      S.sidx = oidx;
      S.sck = ock;
      S.sseg = sseg;
      S.fallback = false;
      S.ties_u = S.u && m == n;  // no dedup: the run boundaries' values stand
      S.all_u = S.ties_u && full_u;  // and every other boundary's
      return;
    }
  }
  uint64_t tie_flags = 1;  // long_run: straight to the full sort
  uint64_t ndup = 0;
  // the 64-bit composite prefixes sorted on their top 32 bits, the keys gathered and the runs
  // of equal prefixes put in order; one sync for the flags (and the caller's check word)
  uint32_t sbu = sb;  // (a forest's hint; 32 if it was short)
  bool made = S.ck_made;
  auto sort_prefix = [&] {
    if (!S.ck_ready && !made) {
      hipLaunchKernelGGL(k_make_ck, GRID(n, BS), dim3(BS), 0, st, (const uint64_t*)K32, seg, sbu, n, ck0, idx0,
                         T.ctr + CTR_TIE, (uint32_t*)rs_scratch);
      LAUNCH_CHECK();
    }
    bool flip = radix_sort_pairs<uint64_t>(ck0, idx0, ck1, idx1, n, S.rs_lo, 64, rs_scratch, st, !S.ck_ready);
    cks = flip ? ck1 : ck0;
    idxs = flip ? idx1 : idx0;
    LAUNCH_CHECK();
    hipLaunchKernelGGL(k_gather, GRID(n, BS), dim3(BS), 0, st, (const uint64_t*)K32, seg, (const uint32_t*)idxs, n,
                       skey, sseg);
    LAUNCH_CHECK();
    hipLaunchKernelGGL(k_tie_fix, GRID(n, BS), dim3(BS), 0, st, (const uint64_t*)cks, n, skey, idxs, sseg, S.kn,
                       T.ctr + CTR_TIE, (uint32_t)S.rs_lo);
    LAUNCH_CHECK();
    if (S.speculate) {  // (element builds: distinct keys, exact segment bits; a long run is read at
                        // the build's first sync, CTR_TIE, and the build redone -- no sync here)
      tie_flags = 0;
      ndup = 0;
      return;
    }
    HIPCHK(hipMemcpyAsync(c->h_pinned + 2, T.ctr + CTR_NDUP, 16, hipMemcpyDeviceToHost, st));  // [2] dups, [3] flags
    if (S.chk) HIPCHK(hipMemcpyAsync(c->h_pinned + 1, S.chk, 8, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    tie_flags = c->h_pinned[3];
    ndup = c->h_pinned[2];
  };
  if (!S.ck_path) {
    sort_prefix();
    if (tie_flags & 4) {  // a trie id past the hinted bits: again with 32
      if (S.ck_ready) throw KhError{KH_EINTERNAL, "sort: segment bits on prepared prefixes"};
      HIPCHK(hipMemsetAsync(T.ctr + CTR_NDUP, 0, 16, st));
      made = false;  // (the prefixes again, with 32 segment bits)
      sbu = 32;
      S.sb = 32;
      S.rs_lo = 32;  // (the segment id alone fills the leading 32 bits)
      sort_prefix();
    }
  }
  const bool fallback = tie_flags & 1, dups = tie_flags & 2;
  uint64_t m = n;
  uint32_t* sidx = idxs;
  if (fallback) {
    // full 256-bit (+segment) LSD sort from the input order
    uint32_t* ia = idx0;
    uint32_t* ib = idx1;
    uint64_t* ka = ck0;
    uint64_t* kb = ck1;
    hipLaunchKernelGGL(k_make_ck, GRID(n, BS), dim3(BS), 0, st, (const uint64_t*)K32, seg, 0u, n, ka, ia,
                       (unsigned long long*)nullptr, (uint32_t*)nullptr);
    LAUNCH_CHECK();
    auto pass = [&](int word, int bits) {
      if (word >= 0)
        hipLaunchKernelGGL(k_word_key, GRID(n, BS), dim3(BS), 0, st, (const uint64_t*)K32, (const uint32_t*)ia, word,
                           n, ka);
      else if (word == -2)
        hipLaunchKernelGGL(k_kn_key, GRID(n, BS), dim3(BS), 0, st, S.kn, (const uint32_t*)ia, n, ka);
      else
        hipLaunchKernelGGL(k_seg_key, GRID(n, BS), dim3(BS), 0, st, seg, (const uint32_t*)ia, n, ka);
      LAUNCH_CHECK();
      if (radix_sort_pairs(ka, ia, kb, ib, n, 0, bits, rs_scratch, st)) {
        std::swap(ka, kb);
        std::swap(ia, ib);
      }
    };
    if (S.kn) pass(-2, 8);  // least significant: the length
    for (int w = 3; w >= 0; --w) pass(w, 64);
    if (segmented) pass(-1, ((sbu + 7) / 8) * 8);
    hipLaunchKernelGGL(k_gather, GRID(n, BS), dim3(BS), 0, st, (const uint64_t*)K32, seg, (const uint32_t*)ia, n,
                       skey, sseg);
    LAUNCH_CHECK();
    sidx = ia;
  }
  if (fallback || dups) {
    // keep the LAST of equal keys (later puts win): flags, scan, compaction.  Without the
    // full sort the count of dropped keys came with the tie flags: no sync of its own, and the
    // scan in multi-block form (a 1024-thread block waited ~90 us for a CU beside a block
    // commit's other phase, profiles/r5m_block_commit_timeline_50m.json)
    uint32_t* keep = (uint32_t*)(sidx == idx0 ? ck1 : ck0);  // n*8 free bytes
    uint32_t* keep_pos = sidx == idx0 ? idx1 : idx0;
    hipLaunchKernelGGL(k_dup, GRID(n, BS), dim3(BS), 0, st, (const uint64_t*)skey, (const uint32_t*)sseg,
                       (const uint32_t*)sidx, S.kn, n, keep);
    LAUNCH_CHECK();
    uint32_t* mtot = (uint32_t*)(T.ctr + CTR_M);
    scan_exclusive<uint32_t>(keep, keep_pos, n, mtot, scan_scratch, st, fallback);
    if (fallback) {
      HIPCHK(hipMemcpyAsync(c->h_pinned, mtot, 4, hipMemcpyDeviceToHost, st));
      HIPCHK(hipStreamSynchronize(st));
      m = (uint32_t)c->h_pinned[0];
    } else {
      m = n - ndup;
    }
    if (m < n) {
      c->ws3.ensure(carve_size({n * 32, n * 4, n * 4}));
      Carver c3{(char*)c->ws3.p, 0, c->ws3.cap};
      uint64_t* skey2 = c3.take<uint64_t>(n * 4);
      uint32_t* sidx2 = c3.take<uint32_t>(n);
      uint32_t* sseg2 = segmented ? c3.take<uint32_t>(n) : nullptr;
      hipLaunchKernelGGL(k_compact, GRID(n, BS), dim3(BS), 0, st, (const uint64_t*)skey, (const uint32_t*)sidx,
                         (const uint32_t*)sseg, (const uint32_t*)keep_pos, (const uint32_t*)keep, n, skey2, sidx2,
                         sseg2);
      LAUNCH_CHECK();
      skey = skey2;
      sidx = sidx2;
      sseg = sseg2;
    }
  }
  S.m = m;
  S.sidx = sidx;
  S.skey = skey;
  S.sseg = sseg;
  S.fallback = fallback;
}

static void build_stats(kh_ctx* c, const unsigned long long* hc, kh_stats* stats);
static void run_build_once(kh_ctx* c, const BuildArgs& A, BuildOut& O, kh_stats* stats);
static void run_build(kh_ctx* c, const BuildArgs& A, BuildOut& O, kh_stats* stats) {
  try {
    run_build_once(c, A, O, stats);
  } catch (SpecRetry&) {
    BuildArgs B = A;
    B.no_spec = true;
    run_build_once(c, B, O, stats);
  }
}
static void run_build_once(kh_ctx* c, const BuildArgs& A, BuildOut& O, kh_stats* stats) {
  hipStream_t st = c->st;
  const uint64_t n = A.n;
  const bool segmented = A.seg != nullptr;
  const uint64_t nres = segmented ? A.nseg : (A.depth0 == 1 ? 16 : 1);
  if (n >= (1ULL << 31)) throw KhError{KH_EINVAL, "n must be < 2^31 per device"};
  if (A.depth0 > 1) throw KhError{KH_EINVAL, "depth0 must be 0 or 1"};
  if (segmented && A.depth0 != 0) throw KhError{KH_EINVAL, "segmented builds use depth0 = 0"};
  if (!(A.flags & KH_HASH_KEYS) && A.klen != 32) throw KhError{KH_EINVAL, "keys must be 32 bytes unless KH_HASH_KEYS"};
  if (A.klen == 0 || A.klen > 4096) throw KhError{KH_EINVAL, "bad key length"};
  const uint32_t sb = segmented ? bits_for(A.nseg) : 0;
  if (sb > 32) throw KhError{KH_EINVAL, "too many segments"};
  // plain root builds hash their leaves on c->st2 while c->st computes the branch
  // topology (trie_ops.h "early leaves"); write-back and incremental builds keep
  // the leaf stage after the topology (they need the parents / dirty marks first)
  const bool early = !A.emit && !A.el && !A.kn;
  if (A.kn && (A.emit || A.el || (A.flags & KH_HASH_KEYS)))
    throw KhError{KH_EINVAL, "variable-length keys: root-only builds of unhashed keys"};
  // Leaf positions (trie_ops.h Topo::lpos; unsegmented plain root builds): no leaf child
  // records at all -- the branch kernels read each leaf child's stash at its sorted position.
  // Segmented early builds reach their parents' child records by a link pass on the topology
  // stream (slot of each sorted leaf) and a copy pass after the join (k_leaf_move).
  const bool lpos = early && !segmented;

  O.res_hash.assign(nres * 4, 0);
  O.res_len.assign(nres, 0);
  O.res_inl.assign(nres * 4, 0);
  if (stats) {
    memset(stats, 0, sizeof(*stats));
    stats->n_inputs = n;
  }
  if (n == 0) return;

  // ---- phase-1 workspace (sized by n)
  const uint64_t nb1 = n;  // boundaries <= n-1; round up
  // keys are moved as 16-byte vectors: caller keys that are not 16-byte aligned get copied
  const bool own_keys = (A.flags & KH_HASH_KEYS) || ((uintptr_t)A.keys & 15);
  std::vector<size_t> sz = {
      own_keys ? n * 32 : 0,                  // K32
      n * 8, n * 8, n * 4, n * 4,             // ck0 ck1 idx0 idx1
      n * 32, segmented ? n * 4 : 0,          // skey sseg
      radix_scratch_bytes(n), scan_scratch_bytes(n, 8),
      nb1, nb1 / 32 + 1024,                   // u, pyramid
      nb1 * 4, nb1 * 4, nb1 * 4, nb1 * 4, nb1, nb1 * 4, nb1, nb1,  // psv nsv pse rep ord isrep glast gk
      nb1 * 4, nb1 * 4, nb1, nb1, nb1 * 4, nb1, nb1 * 4, nb1 * 8, nb1 * 4, nb1 * 4,  // branches
      n * 4, n, n, n * 8, n * 4, n * 8, n * 4,  // leaves, svoff, svlen
      A.emit ? n * 32 : 0, A.emit ? nb1 * 32 : 0, A.emit ? nb1 * 32 : 0,  // hashes
      nres * 32, nres * 4, nres * 32,         // results
      CTR_N * CTR_SHARDS * 8, 64 * 4, 80 * 4, 64 * 4, NBUCKET * ((nb1 + LV_TILE - 1) / LV_TILE) * 4, nb1 * 4,  // ctr hist lb bcnt order
      early ? n * 32 : 0, early ? n : 0, early ? n * 8 : 0,  // early leaves: stashed references, meta, pd|position
      early && !lpos ? n * 8 : 0,                                 // link slots (segmented early builds)
      A.kn ? n : 0,                           // sorted key lengths
      nb1 * 4, nb1 * 4, nb1 * 4, nb1, nb1, nb1,  // branch tables in key-order ids (BrTab J)
      lpos ? nb1 * 4 : 0, lpos ? nb1 * 4 : 0, lpos ? n * 4 : 0,  // leaf positions: range ends (J, T), long list
      nb1 * 4, nb1 * 4,                       // tile topology: boundaries left to the whole-array ANSV / chain
  };
  c->ws1.ensure(carve_size(sz));
  Carver cv{(char*)c->ws1.p, 0, c->ws1.cap};
  uint64_t* K32 = own_keys ? cv.take<uint64_t>(n * 4) : (uint64_t*)A.keys;
  uint64_t* ck0 = cv.take<uint64_t>(n);
  uint64_t* ck1 = cv.take<uint64_t>(n);
  uint32_t* idx0 = cv.take<uint32_t>(n);
  uint32_t* idx1 = cv.take<uint32_t>(n);
  uint64_t* skey = cv.take<uint64_t>(n * 4);
  uint32_t* sseg = segmented ? cv.take<uint32_t>(n) : nullptr;
  void* rs_scratch = cv.take<char>(radix_scratch_bytes(n));
  void* scan_scratch = cv.take<char>(scan_scratch_bytes(n, 8));
  Topo T{};
  T.u = cv.take<uint8_t>(nb1);
  uint8_t* pyr = cv.take<uint8_t>(nb1 / 32 + 1024);
  T.psv = cv.take<int32_t>(nb1);
  T.nsv = cv.take<int32_t>(nb1);
  T.pse = cv.take<int32_t>(nb1);
  T.rep = cv.take<uint32_t>(nb1);
  T.ord = cv.take<uint8_t>(nb1);
  T.isrep_bid = cv.take<uint32_t>(nb1);
  T.glast = cv.take<uint8_t>(nb1);
  T.gk = cv.take<uint8_t>(nb1);
  T.br_k = cv.take<uint32_t>(nb1);
  T.br_cbase = cv.take<uint32_t>(nb1);
  T.br_depth = cv.take<uint8_t>(nb1);
  T.br_ext = cv.take<uint8_t>(nb1);
  T.br_parent = cv.take<uint32_t>(nb1);
  T.br_pord = cv.take<uint8_t>(nb1);
  T.br_first = cv.take<uint32_t>(nb1);
  T.br_aoff = cv.take<uint64_t>(nb1);
  T.br_len = cv.take<uint32_t>(nb1);
  T.ex_len = cv.take<uint32_t>(nb1);
  T.lf_parent = cv.take<uint32_t>(n);
  T.lf_pord = cv.take<uint8_t>(n);
  T.lf_pd = cv.take<int8_t>(n);
  T.lf_aoff = cv.take<uint64_t>(n);
  T.lf_len = cv.take<uint32_t>(n);
  T.svoff = cv.take<uint64_t>(n);
  T.svlen = cv.take<uint32_t>(n);
  T.lf_hash = A.emit ? cv.take<uint64_t>(n * 4) : nullptr;
  T.br_hash = A.emit ? cv.take<uint64_t>(nb1 * 4) : nullptr;
  T.ex_hash = A.emit ? cv.take<uint64_t>(nb1 * 4) : nullptr;
  T.res_hash = cv.take<uint64_t>(nres * 4);
  T.res_len = cv.take<uint32_t>(nres);
  T.res_inl = cv.take<uint64_t>(nres * 4);
  T.ctr = cv.take<unsigned long long>(CTR_N * CTR_SHARDS);
  T.depth_hist = cv.take<uint32_t>(64);
  uint32_t* lb = cv.take<uint32_t>(80);
  uint32_t* wcnt = cv.take<uint32_t>(64);  // k_branch_wide: the wide branches of each level (zeroed below)
  const uint32_t nblk_max = (uint32_t)((nb1 + LV_TILE - 1) / LV_TILE);
  uint32_t* bcnt = cv.take<uint32_t>((uint64_t)NBUCKET * nblk_max);
  uint32_t* order = cv.take<uint32_t>(nb1);
  T.lf_eref = early ? cv.take<uint64_t>(n * 4) : nullptr;
  T.lf_emeta = early ? cv.take<uint8_t>(n) : nullptr;
  T.pdinv = early ? cv.take<uint64_t>(n) : nullptr;
  T.lf_dst = early && !lpos ? cv.take<uint64_t>(n) : nullptr;
  T.kin = K32;
  uint8_t* skn = A.kn ? cv.take<uint8_t>(n) : nullptr;
  BrTab J{};
  J.k = cv.take<uint32_t>(nb1);
  J.parent = cv.take<uint32_t>(nb1);
  J.first = cv.take<uint32_t>(nb1);
  J.depth = cv.take<uint8_t>(nb1);
  J.ext = cv.take<uint8_t>(nb1);
  J.pord = cv.take<uint8_t>(nb1);
  if (lpos) {
    J.end = cv.take<uint32_t>(nb1);
    T.br_end = cv.take<uint32_t>(nb1);
    T.longlist = cv.take<uint32_t>(n);
    T.lpos = 1;
  }
  uint32_t* tlist_a = cv.take<uint32_t>(nb1);
  uint32_t* tlist_c = cv.take<uint32_t>(nb1);
  T.depth0 = A.depth0;
  T.segmented = segmented ? 1 : 0;
  T.vals = A.vals;
  T.voff = A.voff;
  T.vlen_in = A.vlen;

  // results, counters, depth histogram and level bounds are carved back to back: one memset
  HIPCHK(hipMemsetAsync(T.res_hash, 0, (size_t)((char*)(wcnt + 64) - (char*)T.res_hash), st));

  // stage events (kh_stats' t_keys / t_sort / t_topo / t_leaf / t_branch): not for a forest's
  // element builds, whose host is the bottleneck (the block-commit HIP API trace: every API
  // call of a commit counts); their stats keep t_total only
  const bool stage_ev = !A.el;
  HIPCHK(hipEventRecord(c->ev[0], st));
  // ---- 1. keys (the plain path takes its 32-bit sort keys from the hashing pass)
  // plain root builds sort 32-bit words (segment id | leading key bits) with the input
  // index and never gather the sorted keys.  Segmented builds too while the key bits left
  // beside the segment id keep runs of equal words short (the block-local tie fix orders
  // them; one longer than TIE_RUN_MAX falls back to the full sort): at most one key per
  // four word values on average.  Otherwise the 64-bit composite sort.
  const bool seg_words_ok = segmented && sb + CK_KEY_BITS <= 32 && (n / A.nseg) <= (1ULL << (32 - sb - 2));
  const bool ck_path = early && !A.kn && (!segmented || seg_words_ok);
  const bool ck_ready = ck_path && (A.flags & KH_HASH_KEYS);
  // hashed keys of an unsegmented build up to 2^20 (a run of equal top-24 bits every 32 keys at
  // most): the words' lowest 8 bits are left to the tie kernel -- one radix pass less
  const uint32_t tsh = ck_ready && !segmented && n <= (1ull << 20) ? 8u : 0u;
  // host inputs still arriving: the hashing of the plain path starts part by part as the keys
  // land; every other path waits for all keys (and the value offsets)
  if (A.hs && !ck_ready) A.hs->stream_wait(st, A.hs->nkp);
  if (ck_ready) {
    uint32_t* c0 = (uint32_t*)ck0;
    const uint32_t parts = A.hs ? A.hs->nkp : 1;
    for (uint32_t p = 0; p < parts; ++p) {
      const uint64_t a = A.hs && p ? A.hs->kend[p - 1] : 0, b = A.hs ? A.hs->kend[p] : n;
      if (A.hs) A.hs->stream_wait(st, p);
      if (A.klen <= 135)
        hipLaunchKernelGGL(k_hash_keys_ck<true>, GRID(b - a, BS), dim3(BS), 0, st, A.keys, A.klen, a, b, K32, c0, idx0,
                           A.seg, sb);
      else
        hipLaunchKernelGGL(k_hash_keys_ck<false>, GRID(b - a, BS), dim3(BS), 0, st, A.keys, A.klen, a, b, K32, c0, idx0,
                           A.seg, sb);
      LAUNCH_CHECK();
    }
  } else if (A.flags & KH_HASH_KEYS) {
    if (A.klen <= 135)
      hipLaunchKernelGGL(k_hash_keys<true>, GRID(n, BS), dim3(BS), 0, st, A.keys, A.klen, n, K32);
    else
      hipLaunchKernelGGL(k_hash_keys<false>, GRID(n, BS), dim3(BS), 0, st, A.keys, A.klen, n, K32);
    LAUNCH_CHECK();
  } else if (own_keys) {
    HIPCHK(hipMemcpyAsync(K32, A.keys, n * 32, hipMemcpyDeviceToDevice, st));
  }
  if (stage_ev) HIPCHK(hipEventRecord(c->ev[1], st));

  // ---- 2. sort + dedup
  // speculative sorts (no sync for the tie kernel's flags): the plain path's 32-bit words, and the
  // element builds' composite sort (a forest commit's elements are distinct keys, their segment
  // bits exact: only a run past the tie kernel, rare, redoes the build)
  const bool spec = (ck_path || (A.el && !A.kn)) && !A.no_spec && c->spec_off == 0;
  if (c->spec_off) --c->spec_off;
  uint64_t m = n;
  uint32_t* sidx = nullptr;
  bool fallback = false;
  bool ties_u = false, all_u = false;
  {
    SortIO S{(const uint64_t*)K32, A.seg, sb, n, ck0, ck1, idx0, idx1, skey, sseg, rs_scratch, scan_scratch, T.ctr,
             A.kn, ck_ready};
    S.ck_path = ck_path;
    S.tsh = tsh;
    // element builds (hashed paths, few per segment): the leading 24 composite bits suffice
    if (A.el && !A.kn && sb <= 18 && (segmented ? n / A.nseg : n) <= (1ull << (19 - (segmented ? sb : 0))))
      S.rs_lo = 40;
    S.speculate = spec;
    S.u = T.u;
    S.depth0 = A.depth0;
    sort_dedup(c, S);
    m = S.m;
    sidx = S.sidx;
    skey = S.skey;
    sseg = S.sseg;
    fallback = S.fallback;
    T.sck = S.sck;  // non-null: no sorted keys materialised (trie_ops.h sorted_key)
    T.ck_sb = S.sck ? sb : 0;
    ties_u = S.ties_u;
    all_u = S.all_u;
  }
  const bool ties = fallback;
  T.m = m;
  T.skey = skey;
  T.sidx = sidx;
  T.sseg = sseg;
  if (early) {  // the leaves read their spans in input order; long ones through sidx
    T.svoff = nullptr;
    T.svlen = nullptr;
  } else {
    if (A.vals_ready) HIPCHK(hipStreamWaitEvent(st, A.vals_ready, 0));
    if (A.hs) A.hs->stream_wait(st, A.hs->nkp + 1);
    if (!A.el) {  // (element builds gather their spans with the element properties below)
      hipLaunchKernelGGL(k_val_gather, GRID(m, BS), dim3(BS), 0, st, T);
      LAUNCH_CHECK();
    }
  }
  if (A.kn) {
    hipLaunchKernelGGL(k_kn_gather, GRID(m, BS), dim3(BS), 0, st, A.kn, (const uint32_t*)sidx, m, skn);
    LAUNCH_CHECK();
    T.kn = skn;
  }
  if (A.el) {  // element build: the element properties in sorted order (the leaf topology reads them)
    ElemArgs& E = *A.el;
    E.out->ensure(carve_size({m, m * 32, m, m, m * 32, m, m * 32, m * 4}));
    Carver ce{(char*)E.out->p, 0, E.out->cap};
    uint8_t* edb = ce.take<uint8_t>(m);
    uint64_t* ebref = ce.take<uint64_t>(m * 4);
    uint8_t* ebrl = ce.take<uint8_t>(m);
    uint8_t* eoldd = ce.take<uint8_t>(m);
    uint64_t* ecref = ce.take<uint64_t>(m * 4);
    uint8_t* ecrl = ce.take<uint8_t>(m);
    T.lf_ref = ce.take<uint64_t>(m * 4);
    T.lf_rlen = ce.take<uint32_t>(m);
    hipLaunchKernelGGL(k_el_gather3, GRID(m, BS), dim3(BS), 0, st, T, E.db, E.bref, E.brl, edb, ebref, ebrl, E.oldd,
                       E.cref, E.crl, eoldd, ecref, ecrl);
    LAUNCH_CHECK();
    T.el_db = edb;
    T.el_bref = ebref;
    T.el_brl = ebrl;
    T.el_oldd = eoldd;
    T.el_cref = ecref;
    T.el_crl = ecrl;
    T.el_late = E.late;
  }
  if (stage_ev) HIPCHK(hipEventRecord(c->ev[2], st));

  // ---- 3. topology
  const uint64_t nb = m - 1;
  unsigned long long* ctr = T.ctr;
  uint32_t* Bp = (uint32_t*)(ctr + CTR_B);
  // (B, br bytes, lf bytes, C, E0, E1: zero since the counter block's memset; the sort uses
  // only CTR_TIE / CTR_M)
  Pyr P{};
  // Grid of the topology kernels that run beside the leaf kernel (early builds): capped at
  // 4 blocks per CU, so they leave the leaf kernel more of the machine and still finish
  // first.  Measured at 100M (profiles/r2zg_cap_ab_100m.json): 46.5 ms against 47.4 uncapped
  // (one thread per element); 2 blocks per CU starve the topology (23.7 ms, step 49.2),
  // 8 per CU slow the leaf kernel (18.8 ms, step 48.5).
  const uint32_t topo_cap = 4u * (uint32_t)c->n_cu;
  auto topo_grid = [&](uint64_t cnt) {
    const uint64_t g = (cnt + BS - 1) / BS;
    return dim3((unsigned)(early && g > topo_cap ? topo_cap : (g ? g : 1)));
  };
  // Early leaves (plain root builds) need only the boundaries: they are hashed in input
  // order on st2 beside the topology.  Their parent depths (and sorted positions) are
  // scattered by the ANSV kernel on st (k_topo_tile, or k_ansv_pd below TOPO_TILE_MIN) and
  // the leaf kernel starts after it (pd_scan); a trie of one key has no topology: a
  // separate k_pd_scatter on st2.  Measured at 100M (profiles/r2y_pd_ab_100m.json): 49.9 ms
  // (in the ANSV) against 52.2 (separate); folded into k_chain 50.6; into k_lcp, the leaf
  // kernel starting right after it, 50.7 (it then runs beside the whole topology: 19.7 ms
  // instead of 14.9).  The later alternatives (the scatter in two passes, before the tile
  // kernel, after it, the leaves in sorted order): DESIGN.md §5.
  const bool pd_scan = early && nb > 0;
  // Tiles from TOPO_TILE_MIN boundaries; below it the extra launches cost more than the
  // dependent loads they save (configs[2] element builds of ~100k: 1.95 against 2.04 ms per
  // block, profiles/r4w_topo_tile_block_ab_50m.json)
  constexpr uint64_t TOPO_TILE_MIN = 1u << 21;
  const bool topo_tile = nb >= TOPO_TILE_MIN;
  // early tile builds keep the representative flags as bits (Topo::rep_bits), in the flag
  // array's own storage (a word per 32 boundaries, every tile's 128 words written by it)
  const bool rbits = early && topo_tile;
  const uint64_t rb_words = rbits ? (nb + TOPO_TILE - 1) / TOPO_TILE * (TOPO_TILE / 32) : 0;
  uint32_t* rb_pref = nullptr;
  if (rbits) {
    T.rep_bits = T.isrep_bid;
    rb_pref = T.isrep_bid + ((rb_words + 63) & ~(uint64_t)63);
    T.rep_pref = rb_pref;
  }
  if (pd_scan) {  // presets for the scatter folded into the ANSV (on st)
    if (m < n) HIPCHK(hipMemsetAsync(T.pdinv, 0xFF, n * 8, st));  // dropped duplicates: PDINV_SKIP
    // every leaf a hash unless it says otherwise (k_topo_tile presets its own tile's leaves)
    if (!topo_tile) HIPCHK(hipMemsetAsync(T.lf_emeta, 32, m, st));
  }
  if (nb > 0) {
    if (all_u)
      hipLaunchKernelGGL(k_lcp_long_runs, dim3((unsigned)std::min<uint64_t>((nb + BS - 1) / BS, 1024)), dim3(BS), 0, st,
                         T, nb, (const unsigned long long*)(ctr + CTR_TIE), tsh, !topo_tile);
    else
      hipLaunchKernelGGL(k_lcp, GRID(nb, BS), dim3(BS), 0, st, T, nb, ties_u,
                         (const unsigned long long*)(ctr + CTR_TIE), spec && !ck_path, !topo_tile);
    LAUNCH_CHECK();
  }
  // host inputs still arriving (A.hs): the leaf launch on st2 waits until the stager has recorded
  // the values' event, so it is enqueued after the topology (which needs no values), behind the
  // first host sync below
  bool leaves_deferred = false;
  auto start_leaves = [&](bool scatter) {  // on st2, after st's work up to ev[8]
    HIPCHK(hipStreamWaitEvent(c->st2, c->ev[8], 0));
    hipStream_t s2 = c->st2;
    if (scatter) {
      if (m < n) HIPCHK(hipMemsetAsync(T.pdinv, 0xFF, n * 8, s2));  // dropped duplicates: PDINV_SKIP
      HIPCHK(hipMemsetAsync(T.lf_emeta, 32, m, s2));  // every leaf a hash unless it says otherwise
      hipLaunchKernelGGL(k_pd_scatter, GRID(m, BS), dim3(BS), 0, s2, T);
      LAUNCH_CHECK();
    }
    if (A.vals_ready) HIPCHK(hipStreamWaitEvent(s2, A.vals_ready, 0));  // the topology need not wait
    if (A.hs) A.hs->stream_wait(s2, A.hs->nkp + 1);
    HIPCHK(hipEventRecord(c->ev[9], s2));
    {
      const uint64_t runs = (n + BS - 1) / BS;
      const uint64_t g = (runs + LEAF_ITEMS - 1) / LEAF_ITEMS;
      hipLaunchKernelGGL(k_leaf_in, dim3((unsigned)std::max<uint64_t>(g, 1)), dim3(BS), 0, s2, T, n);
    }
    LAUNCH_CHECK();
    HIPCHK(hipEventRecord(c->ev[10], s2));
  };
  auto launch_leaves = [&](bool scatter) {  // on st2, after everything enqueued on st so far
    HIPCHK(hipEventRecord(c->ev[8], st));
    if (A.hs && scatter == false)
      leaves_deferred = true;
    else
      start_leaves(scatter);
  };
  if (early && !pd_scan) launch_leaves(true);
  if (nb > 0) {
    P.lv[0] = T.u;
    P.sz[0] = nb;
    P.nl = 1;
    uint8_t* pp = pyr;
    while (P.sz[P.nl - 1] > 64) {
      if (P.nl >= 8) throw KhError{KH_EINTERNAL, "pyramid too deep"};
      uint64_t nin = P.sz[P.nl - 1], nout = (nin + 63) / 64;
      P.lv[P.nl] = pp;
      P.sz[P.nl] = nout;
      P.nl++;
      pp += (nout + 255) & ~(uint64_t)255;
    }
    auto pyramid = [&](int from) {  // (from 2: the tile kernel wrote level 1)
      if (P.nl > from) {  // the levels in one launch (the last block to finish the first does the rest),
                          // after a launch per level while the next one is too big for one block
                          // (100M keys: level 2 has 24k entries, ~0.9 ms for a lone block)
        for (; from + 1 < P.nl && P.sz[from + 1] > 4 * BS; ++from) {
          hipLaunchKernelGGL(k_pyramid, GRID(P.sz[from], BS), dim3(BS), 0, st, P, from, (unsigned int*)nullptr);
          LAUNCH_CHECK();
        }
        hipLaunchKernelGGL(k_pyramid, GRID(P.sz[from], BS), dim3(BS), 0, st, P, from, (unsigned int*)(ctr + CTR_PYR));
        LAUNCH_CHECK();
      }
    };
    // (k_topo_tile presets its own tile's boundaries; below it k_lcp / k_lcp_long_runs do)
    if (topo_tile) {
      // ANSV and chains tile by tile in LDS (k_topo_tile, the early leaves' parent depths with
      // them); the leaves start right after it; the few boundaries whose answers leave their
      // tile (k_ansv_list / k_chain_list over the whole pyramid) run beside the leaves
      unsigned long long* tcnt = ctr + CTR_TLIST;
      hipLaunchKernelGGL(k_topo_tile, dim3((unsigned)((nb + TOPO_TILE - 1) / TOPO_TILE)), dim3(TT_THREADS), 0, st, T,
                         nb, pd_scan, tcnt, tlist_a, tlist_c, P.nl > 1 ? (uint8_t*)P.lv[1] : (uint8_t*)nullptr);
      LAUNCH_CHECK();
      if (pd_scan) launch_leaves(false);
      pyramid(2);
      hipLaunchKernelGGL(k_ansv_list, topo_grid(nb / 16 + 1), dim3(BS), 0, st, T, P, (const uint32_t*)tlist_a,
                         (const unsigned long long*)tcnt);
      hipLaunchKernelGGL(k_chain_list, topo_grid(nb / 16 + 1), dim3(BS), 0, st, T, (const uint32_t*)tlist_c,
                         (const unsigned long long*)(tcnt + 1));
      LAUNCH_CHECK();
    } else {
      pyramid(1);
      if (pd_scan)
        hipLaunchKernelGGL(k_ansv_pd, GRID(m, BS), dim3(BS), 0, st, T, P, nb);
      else
        hipLaunchKernelGGL(k_ansv, GRID(nb, BS), dim3(BS), 0, st, T, P, nb);
      LAUNCH_CHECK();
      if (pd_scan) launch_leaves(false);
      hipLaunchKernelGGL(k_chain, topo_grid(nb), dim3(BS), 0, st, T, nb);
      LAUNCH_CHECK();
    }
    if (rbits) {  // branch ids: the prefix of the bit words' popcounts
      hipLaunchKernelGGL(k_rep_popc, topo_grid(rb_words), dim3(BS), 0, st, (const uint32_t*)T.rep_bits, rb_words,
                         rb_pref);
      LAUNCH_CHECK();
      scan_exclusive<uint32_t>(rb_pref, rb_pref, rb_words, Bp, scan_scratch, st);
    } else {
      scan_exclusive<uint32_t>(T.isrep_bid, T.isrep_bid, nb, Bp, scan_scratch, st);
    }
    // branch tables in key-order ids first (k_branch_topo writes them, thread per boundary)
    Topo TJ = T;
    TJ.br_k = J.k;
    TJ.br_parent = J.parent;
    TJ.br_first = J.first;
    TJ.br_depth = J.depth;
    TJ.br_ext = J.ext;
    TJ.br_pord = J.pord;
    TJ.br_end = J.end;
    hipLaunchKernelGGL(k_branch_topo, topo_grid(nb), dim3(BS), 0, st, TJ, P, nb);
    LAUNCH_CHECK();
    // level order (grids sized by nb; threads past B exit), then every branch id
    // becomes its level position
    const uint32_t nblk = (uint32_t)((nb + LV_TILE - 1) / LV_TILE);  // (the host's bound; the device's is B's)
    uint32_t* ncnt = lb + 72;
    hipLaunchKernelGGL(k_level_count, dim3(nblk), dim3(BS), 0, st, TJ, (const uint32_t*)Bp, bcnt, ncnt);
    LAUNCH_CHECK();
    // (a small table: one block scans the bound's entries, those past the device's count unread later)
    const uint64_t nbt = (uint64_t)NBUCKET * nblk;
    scan_exclusive<uint32_t>(bcnt, bcnt, nbt, (uint32_t*)nullptr, scan_scratch, st, true,
                             nbt > SCAN_SMALL_MAX ? (const uint32_t*)ncnt : nullptr);
    hipLaunchKernelGGL(k_level_scatter, dim3(nblk), dim3(BS), 0, st, TJ, (const uint32_t*)Bp,
                       (const uint32_t*)bcnt, order);
    LAUNCH_CHECK();
    hipLaunchKernelGGL(k_level_bounds, dim3(1), dim3(64), 0, st, (const uint32_t*)bcnt, (const uint32_t*)Bp, lb);
    LAUNCH_CHECK();
    hipLaunchKernelGGL(k_branch_permute, topo_grid(nb), dim3(BS), 0, st, T, J, (const uint32_t*)order,
                       (const uint32_t*)Bp);
    LAUNCH_CHECK();
    if (lpos || rbits) {  // (leaf positions: only the few long and top leaves resolve a parent later;
                          // segmented early builds' leaf links do, one more lookup each: through the
                          // order itself, not a 100M-boundary remap pass beside the leaf kernel)
      T.bid_pos = order;
    } else {
      hipLaunchKernelGGL(k_bid_remap, topo_grid(nb), dim3(BS), 0, st, T, (const uint32_t*)order, nb);
      LAUNCH_CHECK();
    }
    // child record bases: the first B entries only (B from the device; no clearing of the
    // entries past it, and a third of the 100M-entry scan's traffic beside the leaf kernel)
    scan_exclusive<uint32_t>(T.br_k, T.br_cbase, nb, (uint32_t*)(ctr + CTR_C), scan_scratch, st, true,
                             (const uint32_t*)Bp);
  }
  if (early && !lpos) {  // the leaves' slots, while they are still being hashed
    hipLaunchKernelGGL(k_leaf_link, topo_grid(m), dim3(BS), 0, st, T);
    LAUNCH_CHECK();
  }
  if (early) {
    HIPCHK(hipEventRecord(c->ev[3], st));  // topology done (the leaves may still run)
  } else {
    hipLaunchKernelGGL(k_leaf_topo, GRID(m, BS), dim3(BS), 0, st, T);
    LAUNCH_CHECK();
  }
  // one host sync for every size the second workspace needs: the counters, the depth
  // histogram and the level bounds are carved back to back, one copy.  Early builds take it
  // while the leaf kernel still runs (the child records are carved and cleared beside it) and
  // read the leaves' own counters (long and inline leaves) with a second, short one
  const size_t tcopy = (size_t)((char*)(lb + 65) - (char*)ctr);
  if (tcopy > 16384) throw KhError{KH_EINTERNAL, "counter block exceeds the pinned staging"};
  HIPCHK(hipMemcpyAsync(c->h_pinned, ctr, tcopy, hipMemcpyDeviceToHost, st));
  HIPCHK(hipStreamSynchronize(st));
  const unsigned long long* hc = c->h_pinned;
  if (spec && hc[CTR_TIE]) {  // repeated keys or a long run after all: redo without speculating
    HIPCHK(hipStreamSynchronize(c->st2));
    c->spec_off = 8;
    throw SpecRetry{};
  }
  if (leaves_deferred) start_leaves(false);
  const uint64_t B = (uint32_t)hc[CTR_B];
  const uint64_t C = (uint32_t)hc[CTR_B + 3];
  if (hc[CTR_ERR]) {  // (the leaves may still run on st2: drained before the workspace is given up)
    HIPCHK(hipStreamSynchronize(c->st2));
    throw KhError{KH_EINTERNAL, hc[CTR_ERR] == ERR_LEAF_TOPO
                                    ? "topology: a boundary value out of range (corrupt topology)"
                                    : "topology invariant violated (group chain > 15)"};
  }
  std::vector<uint32_t> lbh(65, 0);
  memcpy(lbh.data(), (const char*)hc + ((char*)lb - (char*)ctr), 65 * 4);
  if (nb == 0) std::fill(lbh.begin(), lbh.end(), 0u);

  // ---- phase-2 workspace: child records + node arena
  // leaf encodings are kept (transposed message slots) for the write-back, element and
  // variable-key builds (the plain root build hashed its leaves in LDS)
  const bool lmsgs = A.emit || A.kn || A.el;
  const uint64_t lmsg_words = lmsgs ? (uint64_t)LEAF_WORDS * m : 0;
  const uint64_t bmsg_words = A.emit ? (uint64_t)BR_WORDS * B : 0, xmsg_words = A.emit ? (uint64_t)EXT_WORDS * B : 0;
  c->ws2.ensure(carve_size({C * 32, C * 2, lmsg_words * 8, bmsg_words * 8, xmsg_words * 8, lpos ? C * 4 : 0}));
  Carver cv2{(char*)c->ws2.p, 0, c->ws2.cap};
  T.cref = cv2.take<uint64_t>(C * 4);
  T.cmeta = cv2.take<uint16_t>(C);
  T.lmsg = lmsgs ? cv2.take<uint64_t>(lmsg_words) : nullptr;
  T.lstride = m;
  if (lpos) {  // a record without CM_BR is a leaf child's: the metas start at zero
    T.cend = cv2.take<uint32_t>(C);
    HIPCHK(hipMemsetAsync(T.cmeta, 0, C * 2, st));
  }
  if (early) {  // the leaves' counters: their long-leaf bytes, long and inline leaves
    HIPCHK(hipStreamWaitEvent(st, c->ev[10], 0));
    HIPCHK(hipMemcpyAsync(c->h_pinned, ctr, (size_t)CTR_N * CTR_SHARDS * 8, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    if (hc[CTR_ERR] == ERR_LEAF_TOPO)
      throw KhError{KH_EINTERNAL, "leaf stage: a parent depth or sorted position out of range (corrupt topology)"};
  }
  const uint64_t lf_bytes = early ? hc[CTR_LONGB] : hc[CTR_B + 2];
  const uint64_t nlong = lpos ? hc[CTR_LONGN] : 0;
  if (lpos) {  // every leaf is hashed by now: is any of them inline?
    unsigned long long ninl = 0;
    for (int sh = 0; sh < CTR_SHARDS; ++sh) ninl += hc[sh * CTR_N + CTR_INLINE];
    T.lf_inline = ninl ? 1 : 0;
  }
  c->ws_arena.ensure(lf_bytes + 64);
  T.arena = (uint8_t*)c->ws_arena.p;  // long leaves
  T.bmsg = A.emit ? cv2.take<uint64_t>(bmsg_words) : nullptr;
  T.xmsg = A.emit ? cv2.take<uint64_t>(xmsg_words) : nullptr;
  T.lb = lb;
  T.wlist = tlist_a;  // (the tile topology's list, free again: >= B entries)
  if (A.el) {  // element build: every capped reference kept for the forest's records
    ElemArgs& E = *A.el;
    E.outb->ensure(carve_size({B * 32, B * 4, B * 32, B * 4}));
    Carver ce{(char*)E.outb->p, 0, E.outb->cap};
    T.br_ref = ce.take<uint64_t>(B * 4);
    T.br_rlen = ce.take<uint32_t>(B);
    T.ex_ref = ce.take<uint64_t>(B * 4);
    T.ex_rlen = ce.take<uint32_t>(B);
    T.emit_sel = nullptr;  // the forest sets its write-back selection after the build
  }
  if (!early && stage_ev) HIPCHK(hipEventRecord(c->ev[3], st));

  // ---- 4. leaves: encode + hash in LDS (root only), or encode into message slots
  //         that the node-set emitter reads back, then hash
  if (early) {  // hashed already: publish into the child records; long leaves now
    if (lpos) {  // leaf positions: only the long leaves' parents and arena slots
      if (nlong) {
        hipLaunchKernelGGL(k_leaf_fix, GRID(nlong, BS), dim3(BS), 0, st, T, nlong);
        LAUNCH_CHECK();
      }
    } else {  // segmented: the stashed references copied into the parents' child records
      hipLaunchKernelGGL(k_leaf_move, GRID(m, BS), dim3(BS), 0, st, T);
      LAUNCH_CHECK();
    }
    if (lf_bytes) {
      hipLaunchKernelGGL(k_leaf_long, GRID(m, BS), dim3(BS), 0, st, T);
      LAUNCH_CHECK();
    }
  } else {  // write-back and element builds: encodings kept in message slots, then hashed
    // element builds: k_leaf_prep also publishes the elements that keep their reference and
    // lists the re-encoded ones (counter CTR_LIST, zero since the build's counter memset),
    // which k_leaf_hash_list hashes in full waves
    unsigned long long* nlist = A.el ? T.ctr + CTR_LIST : nullptr;
    uint32_t* list = nullptr;
    // late values still to come: the other leaves first, the late ones after them (when they are
    // on the device already, one pass: a second costs ~60 us of latency)
    const bool split = A.el && T.el_late && !(A.late_ready && A.late_ready());
    if (A.el) {
      c->ws_list.ensure(carve_size({m * 4, split ? m * 4 : 0}));
      list = (uint32_t*)c->ws_list.p;
    }
    const uint64_t lblocks = std::max<uint64_t>(std::min<uint64_t>((uint64_t)c->n_cu * 4, (m + BS - 1) / BS), 1);
    if (split) {
      hipLaunchKernelGGL(k_leaf_prep, GRID(m, BS), dim3(BS), 0, st, T, list, nlist, 1, list + m, T.ctr + CTR_LIST2);
      hipLaunchKernelGGL(k_leaf_hash_list, dim3((unsigned)lblocks), dim3(BS), 0, st, T, (const uint32_t*)list,
                         (const unsigned long long*)nlist);
      LAUNCH_CHECK();
    }
    if (A.before_leaves) A.before_leaves();  // (a block commit's account values arrive here)
    hipLaunchKernelGGL(k_leaf_prep, GRID(m, BS), dim3(BS), 0, st, T, list, nlist, split ? 2 : 0, list + m,
                       T.ctr + CTR_LIST2);
    LAUNCH_CHECK();
    if (split) {  // (the late leaves were hashed by the pass itself)
    } else if (A.el) {  // the re-encoded elements hashed from the list
      hipLaunchKernelGGL(k_leaf_hash_list, dim3((unsigned)lblocks), dim3(BS), 0, st, T, (const uint32_t*)list,
                         (const unsigned long long*)nlist);
    } else {
      hipLaunchKernelGGL(k_leaf_hash, GRID(m, BS), dim3(BS), 0, st, T);
    }
    LAUNCH_CHECK();
  }
  if (stage_ev) HIPCHK(hipEventRecord(c->ev[4], st));

  // ---- 5. branch levels, deepest first: encode (gathers the children's refs), then hash
  uint32_t levels = 0;
  // levels of at most XL_LEVEL branches: k_branch_xl (32 lanes per branch, the permutation
  // spread over them); of at most SMALL_LEVEL: k_branch_small (every child record loaded at
  // once); larger ones k_branch_fused (one thread per branch)
  for (int d = 63; d >= 0; --d) {
    uint32_t cnt = lbh[d + 1] - lbh[d];
    if (!cnt) continue;
    if (A.emit) {  // the write-back build keeps every encoding in its message slot for emission
      hipLaunchKernelGGL(k_branch_prep, GRID(cnt, BS), dim3(BS), 0, st, T, (uint64_t)lbh[d], (uint64_t)cnt);
      LAUNCH_CHECK();
      hipLaunchKernelGGL(k_branch_hash, GRID(cnt, BS), dim3(BS), 0, st, T, (uint64_t)lbh[d], (uint64_t)cnt);
    } else {
      const bool small = !A.kn && cnt <= SMALL_LEVEL;
      // (leaf positions, a small level: k_branch_xl / k_branch_small read the leaf children's
      // stashes themselves, as op_leaf_children restates -- a separate pass writing the level's leaf
      // child records first cost 5-12 us + a launch per level)
      if (A.kn)
        hipLaunchKernelGGL(k_branch_fused<0>, GRID(cnt, BS), dim3(BS), 0, st, T, (uint64_t)lbh[d], (uint64_t)cnt);
      else if (small && cnt <= XL_LEVEL)
        hipLaunchKernelGGL(k_branch_xl, dim3((unsigned)((cnt + 1) / 2)), dim3(64), 0, st, T, (uint64_t)lbh[d],
                           (uint64_t)cnt);
      else if (small)
        hipLaunchKernelGGL(k_branch_small, dim3((unsigned)((cnt + SMALL_BPB - 1) / SMALL_BPB)), dim3(64), 0, st, T, (uint64_t)lbh[d],
                           (uint64_t)cnt);
      else if (T.cend) {  // leaf children from their stashes
        Topo TL = T;
        TL.lvl_depth = (uint32_t)d;
        TL.lvl_nsh = 28 - 4 * ((uint32_t)d & 7);
        TL.wcnt = wcnt + d;  // (zeroed with the counters; one per level)
        const dim3 wg((unsigned)std::min<uint64_t>((cnt + BS - 1) / BS, 4u * (uint32_t)c->n_cu));
        if (pos_level_ok(T, (uint32_t)d)) {
          hipLaunchKernelGGL(k_branch_fused<4>, GRID(cnt, BS), dim3(BS), 0, st, TL, (uint64_t)lbh[d], (uint64_t)cnt);
          hipLaunchKernelGGL(k_branch_wide<4>, wg, dim3(BS), 0, st, TL);
        } else {
          hipLaunchKernelGGL(k_branch_fused<6>, GRID(cnt, BS), dim3(BS), 0, st, TL, (uint64_t)lbh[d], (uint64_t)cnt);
          hipLaunchKernelGGL(k_branch_wide<6>, wg, dim3(BS), 0, st, TL);
        }
      } else {
        hipLaunchKernelGGL(k_branch_fused<2>, GRID(cnt, BS), dim3(BS), 0, st, T, (uint64_t)lbh[d], (uint64_t)cnt);
      }
    }
    LAUNCH_CHECK();
    ++levels;
  }
  HIPCHK(hipEventRecord(c->ev[5], st));

  // ---- results
  c->T = T;
  c->last_B = B;
  c->last_nres = nres;
  BuildInfo& bi = c->binfo;
  bi.n = n;
  bi.m = m;
  bi.B = B;
  bi.key_perms = (A.flags & KH_HASH_KEYS) ? n * (uint64_t)(A.klen / 136 + 1) : 0;
  bi.arena = lmsg_words * 8 + lf_bytes + (bmsg_words + xmsg_words) * 8;  // node RLP kept in HBM
  bi.levels = levels;
  bi.full_sort = ties;
  bi.early = early;
  bi.stage_ev = stage_ev;
  // A.dev_results (a forest's element build): the results stay on the device and the caller
  // reads the counters at its own next sync (build_stats) -- one host round trip less
  if (A.dev_results) return;
  // through pinned staging: device-to-host copies into pageable memory pin its pages on
  // every call (measured: 20-30 ms per build for 100k roots, scripts/storage_wall_probe.py).
  // The results and the counters are carved back to back: one copy.
  const size_t o_len = (size_t)((char*)T.res_len - (char*)T.res_hash);
  const size_t o_inl = (size_t)((char*)T.res_inl - (char*)T.res_hash);
  const size_t o_ctr = (size_t)((char*)ctr - (char*)T.res_hash);
  uint8_t* hr = pinned_stage(c, o_ctr + CTR_N * CTR_SHARDS * 8);
  HIPCHK(hipMemcpyAsync(hr, T.res_hash, o_ctr + CTR_N * CTR_SHARDS * 8, hipMemcpyDeviceToHost, st));
  HIPCHK(hipStreamSynchronize(st));
  memcpy(O.res_hash.data(), hr, nres * 32);
  memcpy(O.res_len.data(), hr + o_len, nres * 4);
  memcpy(O.res_inl.data(), hr + o_inl, nres * 32);
  build_stats(c, (const unsigned long long*)(hr + o_ctr), stats);
}

// The counters of the last build (host copy hc of T.ctr) -> kh_stats; throws on a device
// invariant flag.  Call once the build's stream work has completed (its events are read).
// the build's counters summed over their shards: hashes, perms, inline, extensions, error
constexpr int BSUM_N = 5;
static void build_stats_sums(kh_ctx* c, const unsigned long long* sums, kh_stats* stats);
static void build_stats(kh_ctx* c, const unsigned long long* hc, kh_stats* stats) {
  unsigned long long sums[BSUM_N] = {0, 0, 0, 0, hc[CTR_ERR]};
  const int idx[4] = {CTR_HASHES, CTR_PERMS, CTR_INLINE, CTR_EXT};
  for (int k = 0; k < 4; ++k)
    for (int r = 0; r < CTR_SHARDS; ++r) sums[k] += hc[r * CTR_N + idx[k]];
  build_stats_sums(c, sums, stats);
}
static void build_stats_sums(kh_ctx* c, const unsigned long long* sums, kh_stats* stats) {
  if (sums[4]) throw KhError{KH_EINTERNAL, "build: device invariant violated"};
  if (!stats) return;
  const BuildInfo& bi = c->binfo;
  stats->n_inputs = bi.n;
  stats->n_leaves = bi.m;
  stats->n_branches = bi.B;
  stats->n_node_hashes = sums[0];
  stats->n_node_perms = sums[1];
  stats->n_inline = sums[2];
  stats->n_extensions = sums[3];
  stats->n_key_perms = bi.key_perms;
  stats->arena_bytes = bi.arena;
  stats->n_levels = bi.levels;
  stats->full_sort = bi.full_sort ? 1 : 0;
  stats->t_total_ms = ev_ms(c->ev[0], c->ev[5]);
  if (!bi.stage_ev) return;
  // split builds: until both halves are hashed (the second half overlaps the first sort)
  stats->t_keys_ms = ev_ms(c->ev[0], c->ev[1]);
  stats->t_sort_ms = ev_ms(c->ev[1], c->ev[2]);
  stats->t_topo_ms = ev_ms(c->ev[2], c->ev[3]);
  // early: the leaf kernel's own span on st2, where it overlaps the topology (the
  // publish of its references runs on st after both; t_total_ms holds it)
  stats->t_leaf_ms = bi.early ? ev_ms(c->ev[9], c->ev[10]) : ev_ms(c->ev[3], c->ev[4]);
  stats->t_branch_ms = ev_ms(c->ev[4], c->ev[5]);
}

// ---------------------------------------------------------------------------
// context management
// ---------------------------------------------------------------------------
static std::mutex g_ctx_mu;
static std::vector<kh_ctx*> g_ctx;

static kh_ctx* ctx_new(int dev) {
  int ndev = 0;
  HIPCHK(hipGetDeviceCount(&ndev));
  if (dev < 0 || dev >= ndev) throw KhError{KH_EDEVICE, "no such device"};
  HIPCHK(hipSetDevice(dev));
  kh_ctx* c = new kh_ctx();
  c->dev = dev;
  // the latency-bound topology kernels (own stream) get the dispatcher's priority
  // over the VALU-bound leaf kernel they overlap with (st2)
  int prio_lo = 0, prio_hi = 0;
  HIPCHK(hipDeviceGetStreamPriorityRange(&prio_lo, &prio_hi));
  HIPCHK(hipDeviceGetAttribute(&c->n_cu, hipDeviceAttributeMultiprocessorCount, c->dev));
  // The topology stream (st) has the priority over the leaf stream (st2): the leaf kernel
  // then shares the CUs with the topology (18 ms instead of 14.7 alone) but the topology
  // stays off the critical path.  Measured (profiles/r2za_*, r2zc_*): the leaf stream first
  // or equal priorities starve the topology (22.3 ms) and cost 0.5 ms;
  // restricting the topology stream to 1/2 or 3/4 of the CUs changes nothing.
  HIPCHK(hipStreamCreateWithPriority(&c->own, hipStreamNonBlocking, prio_hi));
  HIPCHK(hipStreamCreateWithPriority(&c->st2, hipStreamNonBlocking, prio_lo));
  c->st = c->own;
  for (auto& e : c->ev) HIPCHK(hipEventCreate(&e));
  HIPCHK(hipHostMalloc((void**)&c->h_pinned, 16384, hipHostMallocDefault));  // >= CTR_N * CTR_SHARDS words
  return c;
}

static kh_ctx* shared_ctx(int dev) {
  std::lock_guard<std::mutex> g(g_ctx_mu);
  if ((int)g_ctx.size() <= dev) g_ctx.resize(dev + 1, nullptr);
  if (!g_ctx[dev]) g_ctx[dev] = ctx_new(dev);
  return g_ctx[dev];
}

static int current_device() {
  int d = 0;
  if (hipGetDevice(&d) != hipSuccess) return 0;
  return d;
}

#define API_TRY(...)                                                    \
  try {                                                                 \
    __VA_ARGS__;                                                        \
    return KH_OK;                                                       \
  } catch (KhError & e) {                                               \
    return set_err(e.code, e.msg);                                      \
  } catch (std::bad_alloc&) {                                           \
    return set_err(KH_ENOMEM, "host allocation failed");                \
  } catch (std::exception & e) {                                        \
    return set_err(KH_EINTERNAL, e.what());                             \
  }

// copy host inputs into the context's staging buffers
struct Staged {
  const uint8_t* keys;
  const uint8_t* vals;
  const uint64_t* voff;
  const uint32_t* seg;
};
static Staged stage_inputs(kh_ctx* c, const uint8_t* keys, uint32_t klen, const uint8_t* vals, const uint64_t* voff,
                           uint64_t n, const std::vector<uint32_t>* seg) {
  uint64_t v0 = voff[0], vbytes = voff[n] - v0;
  c->in_keys.ensure(n * klen + 64);
  c->in_vals.ensure(vbytes + 64);
  c->in_voff.ensure((n + 1) * 8 + 64);
  std::vector<uint64_t> rel(voff, voff + n + 1);
  for (auto& x : rel) x -= v0;
  hipStream_t st = c->st;
  if (n && klen) HIPCHK(hipMemcpyAsync(c->in_keys.p, keys, n * klen, hipMemcpyHostToDevice, st));
  if (vbytes) HIPCHK(hipMemcpyAsync(c->in_vals.p, vals + v0, vbytes, hipMemcpyHostToDevice, st));
  HIPCHK(hipMemcpyAsync(c->in_voff.p, rel.data(), (n + 1) * 8, hipMemcpyHostToDevice, st));
  const uint32_t* dseg = nullptr;
  if (seg) {
    c->in_seg.ensure(n * 4 + 64);
    if (n) HIPCHK(hipMemcpyAsync(c->in_seg.p, seg->data(), n * 4, hipMemcpyHostToDevice, st));
    dseg = (const uint32_t*)c->in_seg.p;
  }
  HIPCHK(hipStreamSynchronize(st));  // `rel` and `seg` are host temporaries
  return Staged{(const uint8_t*)c->in_keys.p, (const uint8_t*)c->in_vals.p, (const uint64_t*)c->in_voff.p, dseg};
}

__global__ void __launch_bounds__(BS) k_voff_rebase(uint64_t* voff, uint64_t n, uint64_t v0) {
  const uint64_t i = (uint64_t)blockIdx.x * BS + threadIdx.x;
  if (i < n) voff[i] -= v0;
}

// bytes host src -> device dst through the context's pinned ring on c->cs (the stager thread)
static void ring_h2d(kh_ctx* c, uint8_t* dst, const uint8_t* src, uint64_t bytes) {
  for (uint64_t off = 0; off < bytes; off += RING_CHUNK) {
    const uint64_t b = std::min<uint64_t>(RING_CHUNK, bytes - off);
    const uint32_t s = c->ring_next++ % RING_SLOTS;
    if (c->ring_busy[s]) HIPCHK(hipEventSynchronize(c->ring_ev[s]));  // its last DMA has read the chunk
    uint8_t* chunk = c->ring + (size_t)s * RING_CHUNK;
    g_copy_pool.copy(chunk, src + off, b);
    HIPCHK(hipMemcpyAsync(dst + off, chunk, b, hipMemcpyHostToDevice, c->cs));
    HIPCHK(hipEventRecord(c->ring_ev[s], c->cs));
    c->ring_busy[s] = true;
  }
}

// Start streaming n host inputs (HostStage): returns the device buffers they land in; the build
// takes H as BuildArgs::hs (or a forest commit its events) and the call's HostStage joins the
// stager before the call returns.  Keys arrive in at most 64 parts.
static Staged stage_host_async(kh_ctx* c, HostStage& H, const uint8_t* keys, uint32_t klen, const uint8_t* vals,
                               const uint64_t* voff, uint64_t n) {
  const uint64_t v0 = voff[0], vbytes = voff[n] - v0;
  if (voff[n] < v0) throw KhError{KH_EINVAL, "voff not monotone"};
  c->in_keys.ensure(n * klen + 64);
  c->in_vals.ensure(vbytes + 64);
  c->in_voff.ensure((n + 1) * 8 + 64);
  if (!c->cs) HIPCHK(hipStreamCreateWithFlags(&c->cs, hipStreamNonBlocking));
  if (!c->ring) {
    HIPCHK(hipHostMalloc((void**)&c->ring, (size_t)RING_SLOTS * RING_CHUNK, hipHostMallocDefault));
    for (auto& e : c->ring_ev) HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  }
  // the copy stream starts after whatever the build stream still has in flight on these buffers
  HIPCHK(hipEventRecord(c->ev[6], c->st));
  HIPCHK(hipStreamWaitEvent(c->cs, c->ev[6], 0));
  // (parts of 1/64 of the keys, at least 64k: a 100M build hashes 1.56M keys a launch as they land)
  const uint64_t per = std::max<uint64_t>((n + 63) / 64, 65536);
  for (uint64_t e = per; ; e += per) {
    H.kend.push_back(std::min(e, n));
    if (e >= n) break;
  }
  H.nkp = (uint32_t)H.kend.size();
  while (c->part_ev.size() < H.nkp + 2) {
    hipEvent_t e;
    HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    c->part_ev.push_back(e);
  }
  if (!c->hworker) c->hworker.reset(new Worker());
  uint8_t* dk = (uint8_t*)c->in_keys.p;
  uint8_t* dv = (uint8_t*)c->in_vals.p;
  uint64_t* doff = (uint64_t*)c->in_voff.p;
  H.posted = true;
  c->hworker->post([c, &H, keys, klen, vals, voff, n, v0, vbytes, dk, dv, doff] {
    try {
      HIPCHK(hipSetDevice(c->dev));
      for (uint32_t p = 0; p < H.nkp; ++p) {
        const uint64_t a = p ? H.kend[p - 1] : 0;
        ring_h2d(c, dk + a * klen, keys + a * klen, (H.kend[p] - a) * klen);
        HIPCHK(hipEventRecord(H.ev(p), c->cs));
        H.publish();
      }
      ring_h2d(c, (uint8_t*)doff, (const uint8_t*)voff, (n + 1) * 8);
      if (v0) hipLaunchKernelGGL(k_voff_rebase, GRID(n + 1, BS), dim3(BS), 0, c->cs, doff, n + 1, v0);
      HIPCHK(hipGetLastError());
      HIPCHK(hipEventRecord(H.ev(H.nkp), c->cs));
      H.publish();
      ring_h2d(c, dv, vals + v0, vbytes);
      HIPCHK(hipEventRecord(H.ev(H.nkp + 1), c->cs));
      H.publish();
    } catch (KhError& e) {
      std::lock_guard<std::mutex> lk(H.mu);
      H.failed = true;
      H.code = e.code;
      H.msg = e.msg;
      H.cv.notify_all();
    } catch (std::exception& e) {
      std::lock_guard<std::mutex> lk(H.mu);
      H.failed = true;
      H.code = KH_EINTERNAL;
      H.msg = e.what();
      H.cv.notify_all();
    }
  });
  return Staged{dk, dv, doff, nullptr};
}

// A commit's host inputs (kh_block_commit_host, the *_apply_host / root_of_host calls: a few MB
// in up to 11 arrays) packed into the context's pinned buffer at the offsets they take in the
// device staging buffer (c->in_block), value offsets rebased while they are packed, and sent
// in ONE DMA.  Round 5 issued a pageable hipMemcpyAsync per array and a host copy of the
// offsets, then synchronised: ~0.8 ms of a configs[2] block through the host entry point.
struct HostPack {
  struct Part {
    const void* src;
    uint64_t bytes, off, v0;  // v0 != ~0: uint64 offsets, rebased by v0 while packed
  };
  std::vector<Part> parts;
  uint64_t total = 0;
  // reserve a part; returns its offset in the staging buffers
  uint64_t add(const void* src, uint64_t bytes, uint64_t v0 = ~0ull) {
    total = (total + 255) & ~(uint64_t)255;
    parts.push_back(Part{src, bytes, total, v0});
    const uint64_t o = total;
    total += bytes + 16;
    return o;
  }
  // copy every part into pinned memory, one DMA to c->in_block on st; returns the device base
  uint8_t* send(kh_ctx* c, hipStream_t st) {
    c->in_block.ensure(total + 256);
    if (!c->pack_ev) HIPCHK(hipEventCreateWithFlags(&c->pack_ev, hipEventDisableTiming));
    if (c->pack_busy) HIPCHK(hipEventSynchronize(c->pack_ev));  // the last pack's DMA has read the buffer
    if (c->h_pack_cap < total + 256) {
      if (c->h_pack) HIPCHK(hipHostFree(c->h_pack));
      c->h_pack = nullptr;
      c->h_pack_cap = 0;
      const size_t cap = (total + 256) * 5 / 4 + (1u << 20);
      HIPCHK(hipHostMalloc((void**)&c->h_pack, cap, hipHostMallocDefault));
      c->h_pack_cap = cap;
    }
    for (const Part& p : parts) {
      if (!p.bytes || !p.src) continue;
      uint8_t* dst = c->h_pack + p.off;
      if (p.v0 == ~0ull) {
        g_copy_pool.copy(dst, p.src, p.bytes);
      } else {
        const uint64_t* o = (const uint64_t*)p.src;
        uint64_t* d = (uint64_t*)dst;
        for (uint64_t i = 0; i < p.bytes / 8; ++i) d[i] = o[i] - p.v0;
      }
    }
    uint8_t* base = (uint8_t*)c->in_block.p;
    if (total) HIPCHK(hipMemcpyAsync(base, c->h_pack, total, hipMemcpyHostToDevice, st));
    HIPCHK(hipEventRecord(c->pack_ev, st));
    c->pack_busy = true;
    return base;
  }
};

// list-trie keys: key of item i of its trie = RLP of the integer index
// (MptListValidator.scala:15-46, BlockGenerator.scala:157-163; RLP.scala integer
// encoding: 0 -> 0x80, 1..127 -> the byte, else 0x80 + n and n big-endian bytes),
// zero-padded to 32 bytes, with its length in nibbles
__global__ void __launch_bounds__(BS) k_list_keys(const uint32_t* seg, const uint64_t* seg_off, uint64_t n,
                                                  uint64_t* K32, uint8_t* kn) {
  uint64_t i = (uint64_t)blockIdx.x * BS + threadIdx.x;
  if (i >= n) return;
  const uint64_t idx = i - (seg_off[seg[i]] - seg_off[0]);
  uint64_t w = 0;
  uint32_t nb;
  if (idx == 0) {
    w = 0x80;
    nb = 1;
  } else if (idx < 0x80) {
    w = idx;
    nb = 1;
  } else {
    uint32_t L = 0;
    for (uint64_t x = idx; x; x >>= 8) ++L;
    w = 0x80 + L;
    for (uint32_t b = 0; b < L; ++b) w |= ((idx >> (8 * (L - 1 - b))) & 0xFF) << (8 * (b + 1));
    nb = L + 1;
  }
  K32[4 * i] = w;
  K32[4 * i + 1] = K32[4 * i + 2] = K32[4 * i + 3] = 0;
  kn[i] = (uint8_t)(2 * nb);
}

// per-item segment id from device segment offsets (binary search; item i of the call is
// input seg_off[0] + i)
__global__ void __launch_bounds__(BS) k_seg_ids(const uint64_t* seg_off, uint64_t nseg, uint64_t n, uint32_t* seg) {
  uint64_t i = (uint64_t)blockIdx.x * BS + threadIdx.x;
  if (i >= n) return;
  const uint64_t x = seg_off[0] + i;
  uint64_t lo = 0, hi = nseg;  // last s with seg_off[s] <= x
  while (hi - lo > 1) {
    const uint64_t mid = (lo + hi) >> 1;
    if (seg_off[mid] <= x) lo = mid; else hi = mid;
  }
  seg[i] = (uint32_t)lo;
}

static std::vector<uint32_t> seg_ids(const uint64_t* seg_off, uint64_t nseg) {
  const uint64_t n = seg_off[nseg] - seg_off[0];
  std::vector<uint32_t> seg(n);
  for (uint64_t s = 0; s < nseg; ++s) {
    if (seg_off[s + 1] < seg_off[s]) throw KhError{KH_EINVAL, "seg_off not monotone"};
    for (uint64_t i = seg_off[s]; i < seg_off[s + 1]; ++i) seg[i - seg_off[0]] = (uint32_t)s;
  }
  return seg;
}

static const uint8_t EMPTY_TRIE_HASH[32] = {0x56, 0xe8, 0x1f, 0x17, 0x1b, 0xcc, 0x55, 0xa6, 0xff, 0x83, 0x45,
                                            0xe6, 0x92, 0xc0, 0xf8, 0x6e, 0x5b, 0x48, 0xe0, 0x1b, 0x99, 0x6c,
                                            0xad, 0xc0, 0x01, 0x62, 0x2f, 0xb5, 0xe3, 0x63, 0xb4, 0x21};

static void copy_root(const BuildOut& O, uint64_t r, uint8_t* out32) {
  if (O.res_len[r] == 0)
    memcpy(out32, EMPTY_TRIE_HASH, 32);
  else
    memcpy(out32, &O.res_hash[4 * r], 32);
}

// ---------------------------------------------------------------------------
// resident forest (forest.h): node records + anchor map +
// value heap in HBM; a commit rebuilds only the nodes on its dirty paths
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(BS) k_f_descend(FOps O, AMap M, Recs R, uint32_t* touched, uint8_t* replaced,
                                                  uint32_t* tlist, unsigned long long* ctr, uint8_t* vbf) {
  const uint64_t o = (uint64_t)blockIdx.x * BS + threadIdx.x;
  // ctr[0] touched list size, [1] replaced leaves, [2] error, [3] refusal, [6] value-only
  // branches made (vbf[o]: op o puts a value-only branch, forest.h VB_DEPTH).  Every op of a commit passes
  // through its trie's top records: the touched flag is read before it is exchanged, so
  // only the first few ops contend for a hot record's atomic (a stale 0 from the vector
  // cache costs one extra exchange, never a wrong mark), and the replacements are counted
  // per wave.  All lanes stay in the loop until the wave is done (the marks are ballots).
  // The ops are sorted by (trie, key), so the lanes of a wave that reach the same record at
  // a step are adjacent: only the first lane of each run reads and exchanges the flag (at the
  // top levels every lane of every wave reaches the same few records, and one atomic per
  // lane serialised there: the block-commit trace's 355 us account descent).
  auto mark = [&](bool want, uint32_t r) {
    const uint32_t rr = want ? r : NONE;
    const uint32_t prev = __shfl_up(rr, 1);
    const bool lead = want && ((threadIdx.x & 63) == 0 || prev != rr);
    bool first = false;
    if (lead && __hip_atomic_load(&touched[r], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0u)
      first = atomicExch(&touched[r], 1u) == 0u;
    const uint64_t slot = wave_claim(&ctr[0], first);
    if (first) tlist[slot] = r;
  };
  const bool live = o < O.n;
  const uint64_t* K = O.key + 4 * (live ? o : 0);
  const uint32_t t = live ? O.trie[o] : 0;
  uint32_t d = 0;
  bool active = live, repl = false, lost = live, vb = false;
  for (int step = 0; step < 70 && __ballot(active); ++step) {
    uint32_t r = NONE;
    bool leaf = false;
    if (active) {
      r = map_find(M, R, t, d, K);
      if (r == NONE) {
        active = lost = false;
      } else {
        const uint32_t db = R.rdb[r];
        leaf = db == EL_LEAF;
        if (leaf) {
          const uint64_t* L = R.key(r);
          if (L[0] == K[0] && L[1] == K[1] && L[2] == K[2] && L[3] == K[3]) {
            replaced[r] = 1;  // keys are unique in the batch: one op per leaf
            repl = true;
            // a put into a leaf whose remaining path is EMPTY (it hangs under a depth-63 branch)
            // makes khipu's value-only branch (forest.h VB_DEPTH)
            vb = d == VB_DEPTH && O.kind[o] == FOP_UPSERT;
          }
          active = lost = false;
        } else if (db == VB_DEPTH) {  // a value-only branch: only its own key reaches it
          const uint64_t* L = R.key(r);
          if (L[0] == K[0] && L[1] == K[1] && L[2] == K[2] && L[3] == K[3]) {
            if (O.kind[o] == FOP_UPSERT) {  // putInBranchNode with an empty key: the new value
              vb = repl = true;
            } else {  // removeFromBranchNode, then fix: "Branch with no subvalues" (MPTException)
              atomicOr(&ctr[3], 1ULL);
            }
          } else {
            r = NONE;  // (cannot happen: another key leaves the extension above it)
          }
          active = lost = false;
        } else if (lcp_nibbles(load_key(K, 0), load_key(R.key(r), 0)) < (int)db) {
          r = NONE;  // diverges in the extension
          active = lost = false;
        } else {
          d = db + 1;
        }
      }
    }
    mark(r != NONE, r);
  }
  wave_count(&ctr[1], repl);
  wave_count(&ctr[6], vb);
  if (live) vbf[o] = vb ? 1 : 0;
  if (lost) ctr[2] = 3;
}
// value-only branches (k_f_descend's vbf): upsert o's element (rank ur[o], its value in the
// heap) becomes the subtree element of its encoding; hashed encodings (>= 32 B) are listed for
// the write-back set (vbl: encoding offset in enc, length; vbh: hash), count in cnt
__global__ void __launch_bounds__(BS) k_f_vb_elems(FOps O, const uint8_t* vbf, const uint32_t* ur, const uint64_t* uoff,
                                                   const uint8_t* heap, Elems E, uint8_t* enc, uint64_t* vbl,
                                                   uint64_t* vbh, unsigned long long* cnt) {
  const uint64_t o = (uint64_t)blockIdx.x * BS + threadIdx.x;
  if (o >= O.n || !vbf[o]) return;
  const uint64_t e = ur[o], eo = uoff[o] + 32 * e;
  const uint32_t L = vb_encode(heap + E.vo[e], E.vl[e], enc + eo);
  uint64_t w[4];
  if (L >= 32) {
    kec256_msg<false>(enc + eo, L, w);
  } else {
    words_of(enc + eo, L, w);
  }
  for (int q = 0; q < 4; ++q) E.bref[4 * e + q] = w[q];
  E.brl[e] = (uint8_t)(L >= 32 ? 32 : L);
  E.db[e] = (uint8_t)VB_DEPTH;
  if (L >= 32) {
    const unsigned long long s = atomicAdd(cnt, 1ULL);
    vbl[2 * s] = eo;
    vbl[2 * s + 1] = L;
    for (int q = 0; q < 4; ++q) vbh[4 * s + q] = w[q];
  }
}

// upsert op o (its rank among the batch's upserts = ur[o]) -> leaf element; value into the heap
// a commit's inputs staged as one batch: 32-byte keys (copy_keys) and trie ids (when given)
__global__ void __launch_bounds__(BS) k_f_inputs(const uint64_t* up_keys, uint64_t nup, const uint64_t* del_keys,
                                                 uint64_t ndel, bool copy_keys, const uint32_t* up_trie,
                                                 const uint32_t* del_trie, uint64_t* K, uint32_t* Tid,
                                                 unsigned long long* zero) {
  const uint64_t o = (uint64_t)blockIdx.x * BS + threadIdx.x;
  if (o < CTR_N) zero[o] = 0;
  if (o >= nup + ndel) return;
  const bool up = o < nup;
  const uint64_t q = up ? o : o - nup;
  if (copy_keys) {
    const uint64_t* src = (up ? up_keys : del_keys) + 4 * q;
    for (int w = 0; w < 4; ++w) K[4 * o + w] = src[w];
  }
  if (up_trie || del_trie) Tid[o] = up ? up_trie[q] : del_trie[q];
}
__device__ __forceinline__ void upsert_elem(const FOps& O, uint64_t o, uint64_t e, uint32_t seg, uint64_t vo,
                                            uint32_t vl, const Elems& E, bool late = false) {
  E.late[e] = late ? 1 : 0;
  for (int q = 0; q < 4; ++q) E.key[4 * e + q] = O.key[4 * o + q];
  E.seg[e] = seg;
  E.db[e] = EL_LEAF;
  for (int q = 0; q < 4; ++q) E.bref[4 * e + q] = 0;
  E.brl[e] = 0;
  E.vo[e] = vo;
  E.vl[e] = vl;
  E.src[e] = NONE;
  E.oldd[e] = EL_NEW;
  for (int q = 0; q < 4; ++q) E.cref[4 * e + q] = 0;
  E.crl[e] = 0;
}
__global__ void __launch_bounds__(BS) k_f_upsert_elems(FOps O, const uint32_t* tries, uint32_t nt, const uint32_t* ur,
                                                       const uint64_t* uoff, Elems E, uint64_t heap_base,
                                                       uint64_t nups, const uint32_t* sidx, const uint32_t* late) {
  uint64_t o = (uint64_t)blockIdx.x * BS + threadIdx.x;
  if (o == 0) *E.n = nups;
  if (o >= O.n || O.kind[o] != FOP_UPSERT) return;
  const uint64_t e = ur[o];
  upsert_elem(O, o, e, seg_of(tries, nt, O.trie[o]), heap_base + uoff[e], (uint32_t)(uoff[e + 1] - uoff[e]), E,
              late && late[sidx[o]] != 0xFFFFFFFFu);
}
// after the counts are known, CG threads per sorted op o: an upsert's value into the heap at
// its offset uoff[o] (the exclusive scan of the upsert lengths over the sorted ops) and that
// offset by upsert rank (uo[ur[o]]; uo[nups] = the total); a new trie's id into the list
// after the counts are known, CG threads per sorted op o: an upsert's value into the heap at
// its offset uoff[o] (the exclusive scan of the upsert lengths over the sorted ops), that
// offset by upsert rank (uo[ur[o]]; uo[nups] = the total), and its leaf element (rank
// ur[o]; E.n = nups: the gather pushes after them); a new trie's id into the list.  The
// segment of an op is its trie's rank in the sorted list: tpos[o] - 1 + tflag[o].
__global__ void __launch_bounds__(BS) k_f_ops_post(FOps O, const uint32_t* sidx, const uint32_t* ur,
                                                   const uint8_t* vals, const uint64_t* voff, const uint64_t* uoff,
                                                   uint64_t* uo, uint64_t nups, uint64_t total, uint8_t* heap,
                                                   uint64_t heap_base, const uint32_t* tflag, const uint32_t* tpos,
                                                   uint32_t* tries, Elems E, bool meta, int copy,
                                                   const uint32_t* late) {
  // meta: the trie list, the offsets by rank, the upserts' leaf elements (no value bytes read);
  // copy: the value bytes into the heap -- 1 all, 2 those not late, 3 the late ones (late[s] !=
  // ~0: kh_block_commit's account bodies that get a storage root; the rest are copied early)
  const uint64_t g = (uint64_t)blockIdx.x * BS + threadIdx.x;
  const uint64_t o = g / CG;
  const uint32_t sub = threadIdx.x % CG;
  if (meta && g == 0) {
    uo[nups] = total;
    *E.n = nups;
  }
  if (o >= O.n) return;
  if (meta && sub == 0 && tflag[o]) tries[tpos[o]] = O.trie[o];
  if (O.kind[o] != FOP_UPSERT) return;
  const uint64_t s = sidx[o];
  const uint64_t vl = voff[s + 1] - voff[s];
  const bool is_late = late && late[s] != 0xFFFFFFFFu;
  if (meta && sub == 0) {
    uo[ur[o]] = uoff[o];
    upsert_elem(O, o, ur[o], tpos[o] + tflag[o] - 1, heap_base + uoff[o], (uint32_t)vl, E, is_late);
  }
  if (copy == 1 || (copy == 2 && !is_late) || (copy == 3 && is_late))
    copy_bytes_group(heap + heap_base + uoff[o], vals + voff[s], vl, sub);
}
// sorted op o: its kind, the flag of a new trie (the segments of the element build), and for
// an upsert its rank flag and value length (the heap copy); one launch over the sorted ops.
// A single-trie commit (segd false) writes its trie ids (0) here too.
__global__ void __launch_bounds__(BS) k_f_prep(const uint32_t* sidx, uint64_t n, uint64_t nup, bool segd,
                                               uint32_t* trie, const uint64_t* voff, uint8_t* kind, uint32_t* tflag,
                                               uint32_t* isup, uint64_t* ulen, unsigned long long* fctr) {
  const uint64_t o = (uint64_t)blockIdx.x * BS + threadIdx.x;
  if (o < 8) fctr[o] = 0;
  if (o >= n) return;
  const uint32_t s = sidx[o];
  const bool up = s < nup;
  kind[o] = up ? FOP_UPSERT : FOP_DELETE;
  if (segd) {
    tflag[o] = (o == 0 || trie[o] != trie[o - 1]) ? 1u : 0u;
  } else {
    trie[o] = 0;
    tflag[o] = o == 0 ? 1u : 0u;
  }
  isup[o] = up ? 1u : 0u;
  ulen[o] = up ? voff[s + 1] - voff[s] : 0;
}
#ifndef KH_GATHER_BS
#define KH_GATHER_BS 1024
#endif
#ifndef KH_GATHER_PER_CU
#define KH_GATHER_PER_CU 2
#endif
constexpr uint32_t GATHER_BS = KH_GATHER_BS;
__global__ void __launch_bounds__(GATHER_BS) k_f_gather(AMap M, Recs R, const uint32_t* touched, const uint8_t* replaced,
                                                 const uint32_t* tlist, const unsigned long long* ntl_p,
                                                 const uint32_t* tries, uint32_t nt, Elems E, unsigned long long* ctr) {
  // one thread per (touched record, child nibble v): the 16 child lookups of an opened
  // branch are independent map probes (dependent HBM round trips), so they run in 16
  // threads instead of one thread's sequence.  The touched count is read on the device
  // (the descent's counter): a grid-stride loop, no host round trip between the descent
  // and the gather.  Whole blocks iterate together, so every lane reaches the claim.
  __shared__ unsigned long long claim[GATHER_BS / 64 + 1];
  const uint64_t ntl = *ntl_p;
  for (uint64_t g0 = (uint64_t)blockIdx.x * GATHER_BS; g0 < ntl * 16; g0 += (uint64_t)gridDim.x * GATHER_BS) {
    const uint64_t g = g0 + threadIdx.x;
    const uint64_t i = g >> 4;
    const uint32_t v = (uint32_t)(g & 15);
    bool want = false;
    uint32_t er = NONE, seg = 0;
    if (i < ntl) {
      // touched is u32 here; forest.h's gather reads it as a flag
      const uint32_t r = tlist[i];
      if (R.rlive[r] == REC_LIVE) {
        const uint32_t t = R.rt[r], db = R.rdb[r];
        seg = seg_of(tries, nt, t);
        if (db == EL_LEAF) {
          want = v == 0 && !replaced[r];
          er = r;
        } else if ((R.rmask[r] >> v) & 1) {
          uint64_t ck[4] = {R.rk[4ull * r], R.rk[4ull * r + 1], R.rk[4ull * r + 2], R.rk[4ull * r + 3]};
          set_nibble(ck, db, v);
          er = map_find(M, R, t, db + 1, ck);
          if (er == NONE) ctr[2] = 4;
          want = er != NONE && !touched[er];
        }
      }
    }
    const uint64_t e = block_claim(E.n, want, claim);  // every thread of the block reaches the claim
    if (want) elem_fill(R, er, seg, E, e);
  }
  // every trie's untouched root record (a trie no op descended through) -- the same loop form
  for (uint64_t s0 = (uint64_t)blockIdx.x * GATHER_BS; s0 < nt; s0 += (uint64_t)gridDim.x * GATHER_BS) {
    const uint64_t s = s0 + threadIdx.x;
    uint32_t r = NONE;
    if (s < nt) {
      const uint64_t zero[4] = {0, 0, 0, 0};
      r = map_find(M, R, tries[s], 0, zero);
      if (r != NONE && touched[r]) r = NONE;
    }
    const uint64_t e = block_claim(E.n, r != NONE, claim);
    if (r != NONE) elem_fill(R, r, (uint32_t)s, E, e);
  }
}

// after the element build (c->T): one new record per branch (+ extension) at base + j,
// and the write-back selection of branch / extension j (node m + 2j, m + 2j + 1): a node
// identical to the one the old version holds at the same anchor is not written back
__global__ void __launch_bounds__(BS) k_f_branch_recs(Topo T, const uint32_t* Bp, const uint32_t* tries, AMap M,
                                                      Recs R, uint64_t base, uint8_t* sel) {
  const uint64_t j = (uint64_t)blockIdx.x * BS + threadIdx.x;
  if (j >= *Bp) return;
  const uint64_t f = T.br_first[j], r = base + j;
  const uint32_t t = tries[T.sseg ? T.sseg[f] : 0];
  const uint32_t db = T.br_depth[j], ext = T.br_ext[j], d = db - ext;
  const uint64_t* K = T.skey + 4 * f;
  const uint32_t brl = T.br_rlen[j] >= 32 ? 32 : T.br_rlen[j];
  const uint32_t xrl = ext ? (T.ex_rlen[j] >= 32 ? 32 : T.ex_rlen[j]) : brl;
  const uint64_t* xr = ext ? T.ex_ref + 4 * j : T.br_ref + 4 * j;
  uint32_t mask = 0;
  for (uint32_t c = 0; c < T.br_k[j]; ++c) mask |= 1u << (T.cmeta[T.br_cbase[j] + c] >> 8);
  RecVal v;
  for (int q = 0; q < 4; ++q) {
    v.k[q] = K[q];
    v.bref[q] = T.br_ref[4 * j + q];
    v.ref[q] = xr[q];
  }
  v.t = t;
  v.d = (uint8_t)d;
  v.db = (uint8_t)db;
  v.mask = (uint16_t)mask;
  v.live = REC_LIVE;
  v.rl = (uint8_t)xrl;
  v.brl = (uint8_t)brl;
  v.vl = 0;
  v.vo = 0;
  rec_store(R.rk.b, r, v);
  const uint32_t old = map_find(M, R, t, d, K);
  bool same_b = false, same_x = false;
  if (old != NONE && R.rdb[old] == db && R.rbrl[old] == brl) {
    same_b = true;
    for (int q = 0; q < 4; ++q) same_b = same_b && R.rbref[4ull * old + q] == T.br_ref[4 * j + q];
    same_x = same_b && R.rrl[old] == xrl;
    for (int q = 0; q < 4; ++q) same_x = same_x && R.rref[4ull * old + q] == xr[q];
  }
  sel[T.m + 2 * j] = same_b ? 0 : 1;
  sel[T.m + 2 * j + 1] = same_x ? 0 : 1;
}
// elements (sorted position i): the source record (src), the flag of a new record (an
// upsert) for the scan of their ids, and the write-back selection: an upsert's leaf, a leaf
// whose anchor moved, and a subtree's new extension (a subtree hanging at its own depth has
// no node of its own)
// The anchor map is touched only where an anchor changes: an element keeping its source
// record at the same anchor (most of them: the untouched children of the opened branches)
// keeps its map slot.  src[i]: the source record to take out of the map (moved, not touched:
// the touched ones go with the touched list), NONE otherwise; rein[i]: the element's record
// is (re)inserted (new, moved, or a touched leaf no op replaced, whose anchor goes with the
// touched list).
__global__ void __launch_bounds__(BS) k_f_elem_flags(Topo T, Elems E, const uint32_t* touched, uint8_t* sel,
                                                     uint32_t* isnew, uint32_t* src, uint8_t* rein) {
  const uint64_t i = (uint64_t)blockIdx.x * BS + threadIdx.x;
  if (i >= T.m) return;
  const uint32_t s = T.sidx[i], a = (uint32_t)(T.lf_pd[i] + 1);
  const uint32_t es = E.src[s];
  const bool moved = es == NONE || E.oldd[s] != a;
  const bool tch = es != NONE && touched[es] != 0;
  src[i] = (moved && es != NONE && !tch) ? es : NONE;
  rein[i] = (moved || tch) ? 1 : 0;
  isnew[i] = es == NONE ? 1u : 0u;
  const bool sub = T.el_db[i] != EL_LEAF;
  sel[i] = (moved && !(sub && T.el_db[i] == a)) ? 1 : 0;
}
// element records: an upsert's new record (id base + rank), or its source record re-anchored
__global__ void __launch_bounds__(BS) k_f_elem_recs(Topo T, Elems E, const uint32_t* tries, const uint32_t* newrank,
                                                    const uint8_t* rein, Recs R, uint64_t base, uint32_t* eid) {
  const uint64_t i = (uint64_t)blockIdx.x * BS + threadIdx.x;
  if (i >= T.m) return;
  const uint32_t s = T.sidx[i], src = E.src[s];
  const uint64_t r = src == NONE ? base + newrank[i] : src;
  eid[i] = rein[i] ? (uint32_t)r : NONE;
  // an element keeping its source record at the same anchor, untouched (most of them: the
  // unchanged children of the opened branches): the record would be rewritten byte for byte
  // (its key, anchor, references and value span are the element's, copied from it)
  if (src != NONE && !rein[i]) return;
  RecVal v;
  for (int q = 0; q < 4; ++q) {
    v.k[q] = T.skey[4 * i + q];
    v.ref[q] = T.lf_ref[4 * i + q];
    v.bref[q] = T.el_bref[4 * i + q];
  }
  v.t = tries[T.sseg ? T.sseg[i] : 0];
  v.d = (uint8_t)(T.lf_pd[i] + 1);
  v.db = T.el_db[i];
  v.mask = src == NONE ? 0 : R.rmask[r];  // a re-anchored subtree keeps its children
  v.live = REC_LIVE;
  const uint32_t L = T.lf_rlen[i];
  v.rl = (uint8_t)(L >= 32 ? 32 : L);
  v.brl = T.el_brl[i];
  v.vl = E.vl[s];
  v.vo = E.vo[s];
  rec_store(R.rk.b, r, v);
}
// map maintenance: delete records' current anchors (two lists in one launch: the touched
// records, then the element sources), mark dead, insert
// (the first list's records -- the touched ones -- also die here: marked dead, flags cleared)
// (mlog, when journaling: entry i = (slot, its old tag, its old record) of the slot this thread
// changed, slot ~0 for none)
__global__ void __launch_bounds__(BS) k_map_delete(AMap M, Recs R, const uint32_t* list, uint64_t n,
                                                   const uint32_t* list2, uint64_t n2, uint32_t* touched,
                                                   uint8_t* replaced, uint64_t* mlog) {
  const uint64_t i = (uint64_t)blockIdx.x * BS + threadIdx.x;
  if (i >= n + n2) return;
  const uint32_t r = i < n ? list[i] : list2[i - n];
  const uint64_t sl = r == NONE ? ~0ULL : map_slot_of(M, R, r);
  if (mlog) {
    mlog[3 * i] = sl;
    if (sl != ~0ULL) {
      mlog[3 * i + 1] = M.tag[sl];
      mlog[3 * i + 2] = r;
    }
  }
  if (r == NONE) return;
  if (sl != ~0ULL) M.tag[sl] = 1;  // tombstone
  if (i < n) {
    R.rlive[r] = REC_DEAD;
    touched[r] = 0;
    replaced[r] = 0;
  }
}
// an aborted commit: the records its descent flagged are left as they were
__global__ void __launch_bounds__(BS) k_f_untouch(const uint32_t* list, uint64_t n, uint32_t* touched,
                                                  uint8_t* replaced) {
  const uint64_t i = (uint64_t)blockIdx.x * BS + threadIdx.x;
  if (i >= n) return;
  touched[list[i]] = 0;
  replaced[list[i]] = 0;
}
// insert records at their anchors: base + i for i < nb, then list[i - nb] for the next n
// (list may be null when n is 0)
// (list entries NONE are skipped; used, when given, counts the inserts that took an empty
// slot: the table's load, live + tombstones)
__global__ void __launch_bounds__(BS) k_map_insert(AMap M, Recs R, uint64_t base, uint64_t nb, const uint32_t* list,
                                                   uint64_t n, unsigned long long* err, unsigned long long* used,
                                                   uint64_t* mlog) {
  const uint64_t i = (uint64_t)blockIdx.x * BS + threadIdx.x;
  bool fresh = false;
  if (i < nb + n) {
    const uint32_t r = i < nb ? (uint32_t)(base + i) : list[i - nb];
    uint64_t ls = ~0ULL, lt = 0, lr = 0;  // the slot taken, its old tag and record (journal)
    if (r != NONE && R.rlive[r] == REC_LIVE) {
      const unsigned long long h = anchor_tag(R.rt[r], R.rd[r], R.key(r));
      bool done = false;
      for (uint64_t s = h & M.mask, k = 0; k <= M.mask; s = (s + 1) & M.mask, ++k) {
        unsigned long long g = M.tag[s];
        if (g > 1) continue;
        const uint32_t orec = M.rec[s];  // an empty / tombstone slot's record changes only with its tag
        if (atomicCAS(&M.tag[s], g, h) == g) {
          M.rec[s] = r;
          fresh = g == 0;
          done = true;
          ls = s;
          lt = g;
          lr = orec;
          break;
        }
      }
      if (!done) *err = 5;  // full table
    }
    if (mlog) {
      mlog[3 * i] = ls;
      mlog[3 * i + 1] = lt;
      mlog[3 * i + 2] = lr;
    }
  }
  if (used) wave_atomic_add(used, fresh ? 1ULL : 0ULL);
}
// journal (versioned commits): the records a commit rewrites in place -- the touched records
// (they die) and the element sources (re-anchored) -- saved whole before the first change, and
// restored by a rollback; 8 lanes per record, one 16-byte word each
__global__ void __launch_bounds__(BS) k_rec_save(const uint8_t* recs, const uint32_t* l1, uint64_t n1, const uint32_t* l2,
                                                 uint64_t n2, uint32_t* jidx, uint8_t* jrec) {
  const uint64_t g = (uint64_t)blockIdx.x * BS + threadIdx.x, i = g >> 3;
  const uint32_t w = (uint32_t)(g & 7);
  if (i >= n1 + n2) return;
  const uint32_t r = i < n1 ? l1[i] : l2[i - n1];
  if (w == 0) jidx[i] = r;
  if (r == NONE) return;
  ((ulonglong2*)(jrec + i * REC_BYTES))[w] = ((const ulonglong2*)(recs + (uint64_t)r * REC_BYTES))[w];
}
__global__ void __launch_bounds__(BS) k_rec_restore(uint8_t* recs, const uint32_t* jidx, const uint8_t* jrec,
                                                    uint64_t n) {
  const uint64_t g = (uint64_t)blockIdx.x * BS + threadIdx.x, i = g >> 3;
  if (i >= n) return;
  const uint32_t r = jidx[i];
  if (r == NONE) return;
  ((ulonglong2*)(recs + (uint64_t)r * REC_BYTES))[g & 7] = ((const ulonglong2*)(jrec + i * REC_BYTES))[g & 7];
}
// undo one map log (the slots of one launch are distinct: a delete tombstones its record's own
// slot, an insert owns the slot its CAS won)
__global__ void __launch_bounds__(BS) k_map_undo(AMap M, const uint64_t* mlog, uint64_t n) {
  const uint64_t i = (uint64_t)blockIdx.x * BS + threadIdx.x;
  if (i >= n) return;
  const uint64_t s = mlog[3 * i];
  if (s == ~0ULL) return;
  M.tag[s] = mlog[3 * i + 1];
  M.rec[s] = (uint32_t)mlog[3 * i + 2];
}
// per touched trie: its new root (segment result), EMPTY when no element remained
// (block 0 also leaves the commit's final flags in tail: the element build's counters summed
// over their shards (hashes, perms, inline, extensions, error; ctr null: none), the map
// insert's error and fresh-slot count -- so the commit's last sync is one copy)
__global__ void k_f_roots(const uint64_t* res_hash, const uint32_t* res_len, uint32_t nt, uint64_t* roots,
                          const unsigned long long* ctr, const unsigned long long* fctr, unsigned long long* tail) {
  if (blockIdx.x == 0 && threadIdx.x < 8) {
    const int idx[5] = {CTR_HASHES, CTR_PERMS, CTR_INLINE, CTR_EXT, CTR_ERR};
    unsigned long long v = 0;
    if (threadIdx.x < 4) {
      if (ctr)
        for (int r = 0; r < CTR_SHARDS; ++r) v += ctr[r * CTR_N + idx[threadIdx.x]];
    } else if (threadIdx.x == 4) {
      v = ctr ? ctr[CTR_ERR] : 0;
    } else if (threadIdx.x < 7) {
      v = fctr[threadIdx.x - 2];  // 5: fctr[3] (map insert error), 6: fctr[4] (fresh slots)
    }
    tail[threadIdx.x] = v;
  }
  const uint32_t s = blockIdx.x * BS + threadIdx.x;
  if (s >= nt) return;
  const uint64_t E[4] = {0xa655cc1b171fe856ULL, 0x6ef8c092e64583ffULL, 0xc0ad6c991be0485bULL, 0x21b463e3b52f6201ULL};
  for (int q = 0; q < 4; ++q) roots[4 * s + q] = res_len && res_len[s] ? res_hash[4 * s + q] : E[q];
}
// block commit: the new storage root of account upsert i's trie into bytes [len-65, len-33)
// of its body (RLP[nonce, balance, stateRoot, codeHash], PV63.scala:46-51)
__global__ void __launch_bounds__(BS) k_inject_roots(uint8_t* vals, const uint64_t* voff, const uint32_t* acct_trie,
                                                     uint64_t n, const uint32_t* tries, uint32_t nt,
                                                     const uint64_t* roots, unsigned long long* err,
                                                     unsigned long long tok) {
  const uint64_t i = (uint64_t)blockIdx.x * BS + threadIdx.x;
  if (i >= n || acct_trie[i] == 0xFFFFFFFFu) return;
  const uint32_t s = seg_of(tries, nt, acct_trie[i]);
  if (s >= nt || tries[s] != acct_trie[i]) return;  // storage unchanged this block
  const uint64_t e = voff[i + 1];
  if (e - voff[i] < 66 || vals[e - 66] != 0xA0 || vals[e - 33] != 0xA0) {
    *err = tok;  // not an account body
    return;
  }
  const uint8_t* rb = (const uint8_t*)(roots + 4 * s);
  for (int q = 0; q < 32; ++q) vals[e - 65 + q] = rb[q];
}

// ---- versioned commits (Ledger.executeBlock flushes a parallel attempt and, when
// its root does not validate, re-executes sequentially from the SAME parent state,
// Ledger.scala:237-271; validateBlockAfterExecution rejects a block, :603-620; TrieAccounts.rootHash
// flushes a COPY, TrieAccounts.scala:73-80).  A savepoint opens an undo journal: every commit
// after it saves the records it rewrites in place and logs the anchor-map slots it changes, so a
// rollback restores the version of the savepoint in O(changed records), not O(resident trie).
// New records, heap bytes and node ids are appended past the savepoint's ends and simply cut off.
struct JSeg {  // one journaled commit: its saved records and map-slot log ranges (entries)
  uint64_t rpos = 0, rn = 0;  // saved records [rpos, rpos + rn) of jidx / jrec
  uint64_t dpos = 0, dn = 0;  // map log: the deletes (tombstones) ...
  uint64_t ipos = 0, in = 0;  // ... and the inserts, 3 words per entry (slot, old tag, old record)
};
struct Savepoint {
  uint64_t rn = 0, heap_n = 0, nleaves = 0, mused = 0, rdead = 0, map_epoch = 0;
  uint8_t root[32] = {};
  std::vector<uint32_t> tries;  // the last commit's touched tries and roots (kh_forest_last_roots)
  std::vector<uint8_t> roots;
  size_t seg0 = 0;              // journal fill at the savepoint
  uint64_t jrec0 = 0, jmap0 = 0;
  bool em_saved = false;        // the write-back set of the savepoint's version, kept when a later
  bool em_valid = false;        // commit replaced it (kh_trie_emit_nodes after a rollback)
  DevBuf em;
  uint64_t em_n = 0, em_bytes = 0;
};
static void swap_buf(DevBuf& a, DevBuf& b) {
  std::swap(a.p, b.p);
  std::swap(a.cap, b.cap);
  std::swap(a.dev, b.dev);
}

struct kh_trie {
  kh_ctx* c = nullptr;     // the context its commits run on (kh_block_commit moves the storage phase for a call)
  kh_ctx* home = nullptr;  // the context it was opened on
  // Handles opened through the host entry points (the shared context: the JVM's tries) run on a
  // private context of their own (priv: streams and workspaces) and serialise on their own
  // mutex, so commits on different handles overlap on the GPU (TxProcessor.scala:28-35 drives
  // tries from many workers; SURVEY §8b: each handle its own HIP stream).  Handles opened on a
  // caller's context run on it and hold its mutex (the caller owns that stream's ordering).
  std::recursive_mutex own_mu;
  std::recursive_mutex* lk = nullptr;  // every call on the handle holds *lk
  kh_ctx* priv = nullptr;
  uint32_t flags = 0;  // KH_HASH_KEYS: the trie's key encoder; KH_EMIT_NODES: keep each commit's write-back set
  bool forest = false;
  uint32_t tid_bits = 0;  // forests: bits of the trie ids committed so far (+ headroom; 0: none yet)
  uint32_t lo24_off = 0;  // commits left without the 24-bit op sort (a run past the tie kernel fell back)
  DevBuf recs, touched, replaced;  // node records (forest.h Recs: 128 B each), per-commit flags
  uint64_t rcap = 0, rn = 0, rdead = 0;
  DevBuf mslots;  // anchor map: 16-byte (tag, record) slots
  uint64_t mcap = 0, mused = 0;
  DevBuf heap;
  uint64_t heap_n = 0;
  uint64_t nleaves = 0;
  uint8_t root[32] = {};
  DevBuf ws, elout, eloutb, em;  // commit scratch, element-build outputs, last write-back set
  DevBuf tlb, ebuf, tbuf, ubuf, selb, merr;  // touched list, elements, trie ids + roots, upsert offsets, selections
  DevBuf gbuf;                                // batched get: keys, records, lengths, scan scratch
  uint64_t em_n = 0, em_bytes = 0;
  bool em_valid = false;
  uint64_t ntl_hint = 0;  // touched records of the last commit (sizes the next element buffer)
  std::vector<uint32_t> tries;  // last commit: touched tries and their roots
  std::vector<uint8_t> roots;
  uint32_t* d_tries = nullptr;  // ... the same on the device (in tbuf; the block commit's injection reads them)
  uint64_t* d_roots = nullptr;
  // versioned commits: open savepoints (innermost last) and the journal of the commits since the
  // outermost one
  std::vector<std::unique_ptr<Savepoint>> sps;
  std::vector<JSeg> jsegs;
  DevBuf jidx, jrec, jmap;  // saved record ids (u32), saved records (128 B), map-slot log (3 u64)
  uint64_t jrec_n = 0, jmap_n = 0;
  uint64_t map_epoch = 0;   // anchor-map rebuilds so far (a rebuild voids the slot log)
  bool flags_dirty = false; // a descent marked records and its commit did not finish
  DevBuf em_spare;          // the write-back buffer a savepoint's saved set rotates with
  // a commit's tail left in flight (forest_commit, no write-back set): its records and anchor
  // map are written after the call returned; pend (pinned) gets the map's error flag and fresh
  // slot count, read by trie_settle before the host next needs them
  hipEvent_t ev_roots = nullptr, pend_ev = nullptr;
  unsigned long long* pend = nullptr;
  bool pend_valid = false, pend_fresh = false;
  // such a tail failed (its anchor map is not trustworthy): every later call refuses the
  // handle (KH_EINTERNAL) except kh_trie_free
  bool broken = false;
  kh_trie() = default;
  kh_trie(const kh_trie&) = delete;
  kh_trie& operator=(const kh_trie&) = delete;
  ~kh_trie() {
    if (ev_roots) (void)hipEventDestroy(ev_roots);
    if (pend_ev) (void)hipEventDestroy(pend_ev);
    if (pend) (void)hipHostFree(pend);
    if (priv) (void)kh_ctx_destroy(priv);
  }
};
// the in-flight tail of the last commit: its map error and fresh slots (before mused is read)
static void trie_settle(kh_trie* h) {
  if (h->broken) throw KhError{KH_EINTERNAL, "handle unusable: an earlier commit's anchor-map update failed"};
  if (!h->pend_valid) return;
  const hipError_t e = hipEventSynchronize(h->pend_ev);
  if (e != hipSuccess || h->pend[0]) {
    h->broken = true;  // sticky: the map may hold part of that commit
    h->pend_valid = false;
    if (e != hipSuccess) throw KhError{KH_EDEVICE, std::string("commit tail: ") + hipGetErrorString(e)};
    throw KhError{KH_EINTERNAL, "anchor map insert failed"};
  }
  h->pend_valid = false;
  if (h->pend_fresh) h->mused += h->pend[1];
}

// every entry point on a resident handle serialises on its home context (khst.h: reentrant)
#define HANDLE_LOCK(h) std::lock_guard<std::recursive_mutex> handle_lock_(*(h)->lk)
// both handles of a block commit: one mutex when they share a context, else both (std::lock:
// no deadlock against another call locking them in the other order)
struct PairLock {
  std::unique_lock<std::recursive_mutex> a, b;
  PairLock(std::recursive_mutex* x, std::recursive_mutex* y) : a(*x, std::defer_lock), b(*y, std::defer_lock) {
    if (x == y)
      a.lock();
    else
      std::lock(a, b);
  }
};

static Recs recs_of(kh_trie* h) {
  return recs_at((uint8_t*)h->recs.p);
}
static AMap map_of(kh_trie* h) { return AMap{{(uint8_t*)h->mslots.p}, {(uint8_t*)h->mslots.p}, h->mcap - 1}; }

// grow a device array, keeping its first `keep` bytes
static void regrow(DevBuf& b, size_t keep, size_t bytes, hipStream_t st) {
  if (bytes <= b.cap) return;
  DevBuf nb;
  nb.ensure(bytes);
  if (keep) HIPCHK(hipMemcpyAsync(nb.p, b.p, keep, hipMemcpyDeviceToDevice, st));
  HIPCHK(hipStreamSynchronize(st));
  b.release();
  b.p = nb.p;
  b.cap = nb.cap;
  nb.p = nullptr;
  nb.cap = 0;
}
static void recs_reserve(kh_trie* h, uint64_t need) {
  if (need <= h->rcap) return;
  hipStream_t st = h->c->st;
  const uint64_t cap = std::max<uint64_t>(need + need / 2, 4096), n = h->rn;
  regrow(h->recs, n * REC_BYTES, cap * REC_BYTES, st);
  regrow(h->touched, n * 4, cap * 4, st);
  regrow(h->replaced, n, cap, st);
  // the new tail: not live, not touched
  HIPCHK(hipMemsetAsync((uint8_t*)h->recs.p + n * REC_BYTES, 0, h->recs.cap - n * REC_BYTES, st));
  HIPCHK(hipMemsetAsync((uint8_t*)h->touched.p + 4 * n, 0, h->touched.cap - 4 * n, st));
  HIPCHK(hipMemsetAsync((uint8_t*)h->replaced.p + n, 0, h->replaced.cap - n, st));
  h->rcap = std::min({h->recs.cap / REC_BYTES, h->touched.cap / 4, h->replaced.cap});
}
__global__ void __launch_bounds__(BS) k_rec_count_live(Recs R, uint64_t n, unsigned long long* cnt) {
  const uint64_t i = (uint64_t)blockIdx.x * BS + threadIdx.x;
  unsigned long long v = (i < n && R.rlive[i] == REC_LIVE) ? 1 : 0;
  v = wave_sum(v);
  if ((threadIdx.x & 63) == 0 && v) atomicAdd(cnt, v);
}
__global__ void __launch_bounds__(BS) k_heap_live(Recs R, uint64_t n, unsigned long long* cnt) {
  const uint64_t i = (uint64_t)blockIdx.x * BS + threadIdx.x;
  unsigned long long v = (i < n && R.rlive[i] == REC_LIVE) ? R.rvl[i] : 0;
  v = wave_sum(v);
  if ((threadIdx.x & 63) == 0 && v) atomicAdd(cnt, v);
}
// (re)build the anchor map with capacity >= 2 * (records + headroom), inserting every live record
static void map_rebuild(kh_trie* h, uint64_t headroom) {
  h->pend_valid = false;  // (the rebuild counts the table afresh; the stream has run the tail by its sync)
  hipStream_t st = h->c->st;
  uint64_t cap = 1024;
  while (cap < 2 * (h->rn + headroom) + 1024) cap <<= 1;
  h->mslots.ensure(cap * 16);
  h->mcap = cap;
  ++h->map_epoch;  // the journal's slot log no longer applies: a rollback rebuilds the map
  HIPCHK(hipMemsetAsync(h->mslots.p, 0, cap * 16, st));
  h->merr.ensure(64);
  unsigned long long* err = (unsigned long long*)h->merr.p;
  HIPCHK(hipMemsetAsync(err, 0, 16, st));
  if (h->rn) {
    hipLaunchKernelGGL(k_map_insert, GRID(h->rn, BS), dim3(BS), 0, st, map_of(h), recs_of(h), (uint64_t)0, h->rn,
                       (const uint32_t*)nullptr, (uint64_t)0, err, (unsigned long long*)nullptr, (uint64_t*)nullptr);
    hipLaunchKernelGGL(k_rec_count_live, GRID(h->rn, BS), dim3(BS), 0, st, recs_of(h), h->rn, err + 1);
  }
  LAUNCH_CHECK();
  HIPCHK(hipMemcpyAsync(h->c->h_pinned, err, 16, hipMemcpyDeviceToHost, st));
  HIPCHK(hipStreamSynchronize(st));
  if (h->c->h_pinned[0]) throw KhError{KH_EINTERNAL, "anchor map rebuild failed"};
  h->mused = h->c->h_pinned[1];
  h->rdead = h->rn - h->mused;
}

// one level of the open-from-store walk: decode every frontier node into a record (a
// leaf, or a branch with the extension above it) and push its children to the next level
__global__ void __launch_bounds__(BS) k_open_level(OItems I, uint64_t ni, OItems N, NStore S, Recs R,
                                                   unsigned long long* rcount, uint64_t rbase, uint32_t trie,
                                                   uint8_t* heap, unsigned long long* heap_n,
                                                   unsigned long long* leaves, unsigned long long* err,
                                                   uint8_t* missing) {
  const uint64_t i = (uint64_t)blockIdx.x * BS + threadIdx.x;
  if (i >= ni) return;
  const uint64_t* h = I.ref + 4 * i;
  const uint8_t* e;
  uint32_t L;
  if (I.rl[i] == 32) {
    const uint64_t p = key_lower_bound(S.hash, S.m, h);
    if (p >= S.m || key_cmp(S.hash + 4 * p, h) != 0) {  // MPTNodeMissingException (MerklePatriciaTrie.scala:534-537)
      if (atomicCAS(err, OPEN_OK, OPEN_MISSING) == OPEN_OK)
        for (int q = 0; q < 32; ++q) missing[q] = (uint8_t)(h[q >> 3] >> (8 * (q & 7)));
      return;
    }
    const uint32_t j = S.idx[p];
    e = S.enc + S.off[j];
    L = (uint32_t)(S.off[j + 1] - S.off[j]);
  } else {
    e = (const uint8_t*)h;
    L = I.rl[i];
  }
  auto bad = [&](unsigned long long code) { atomicCAS(err, OPEN_OK, code); };
  RItem top;
  if (!rlp_valid(e, L, 0, 0) || !rlp_at(e, L, 0, top) || !top.list) return bad(OPEN_BAD);
  RItem it[18];
  const int k = rlp_items(e, L, top, it, 18);
  const uint32_t a = I.a[i], d = I.d[i];
  uint64_t own[4];  // the node's capped reference (Node.capped, Node.scala:114)
  uint32_t ownl;
  if (L >= 32) {
    for (int q = 0; q < 4; ++q) own[q] = h[q];  // referenced by hash (a root < 32 B: its bytes below)
    ownl = 32;
  } else {
    words_of(e, L, own);
    ownl = L;
  }
  if (L >= 32 && I.rl[i] != 32) return bad(OPEN_BAD);  // an embedded node must be < 32 B
  const uint64_t* pre = I.pre + 4 * i;
  auto push = [&](const uint64_t* np, uint32_t na, uint32_t nd, const uint8_t* cref, uint32_t crl, bool is_hash,
                  const uint64_t* pr, uint32_t prl) {
    const unsigned long long t = atomicAdd(N.n, 1ULL);
    if (t >= N.cap) return bad(OPEN_BAD);
    for (int q = 0; q < 4; ++q) N.pre[4 * t + q] = np[q];
    N.a[t] = (uint8_t)na;
    N.d[t] = (uint8_t)nd;
    uint64_t w[4];
    words_of(cref, crl, w);
    for (int q = 0; q < 4; ++q) N.ref[4 * t + q] = w[q];
    N.rl[t] = (uint8_t)(is_hash ? 32 : crl);
    for (int q = 0; q < 4; ++q) N.pref[4 * t + q] = pr ? pr[q] : w[q];
    N.prl[t] = (uint8_t)(pr ? prl : (is_hash ? 32 : crl));
  };
  if (k == 17) {  // branch [ref_0 .. ref_15, value]
    if (it[16].list || it[16].len) {
      // a secure trie stores a branch value only in khipu's value-only branch (forest.h VB_DEPTH):
      // no children, at depth 64
      bool none = !it[16].list && d == VB_DEPTH;
      for (int c = 0; c < 16 && none; ++c) none = !it[c].list && it[c].len == 0;
      if (!none) return bad(OPEN_VALUE);
      const uint64_t vo = atomicAdd(heap_n, (unsigned long long)it[16].len);
      for (uint32_t q = 0; q < it[16].len; ++q) heap[vo + q] = e[it[16].off + q];
      const uint64_t r = rbase + atomicAdd(rcount, 1ULL);
      for (int q = 0; q < 4; ++q) {
        R.rk[4 * r + q] = pre[q];
        R.rbref[4 * r + q] = own[q];
        R.rref[4 * r + q] = I.pref[4 * i + q];
      }
      R.rt[r] = trie;
      R.rd[r] = (uint8_t)a;
      R.rdb[r] = (uint8_t)VB_DEPTH;
      R.rvo[r] = vo;
      R.rvl[r] = it[16].len;
      R.rbrl[r] = (uint8_t)ownl;
      R.rrl[r] = I.prl[i];
      R.rmask[r] = 0;
      R.rlive[r] = REC_LIVE;
      atomicAdd(leaves, 1ULL);  // (its key counts as one of the trie's keys)
      return;
    }
    uint32_t mask = 0;
    for (int c = 0; c < 16; ++c) {
      if (!it[c].list && it[c].len == 0) continue;
      if (!it[c].list && it[c].len != 32) return bad(OPEN_BAD);
      uint64_t np[4] = {pre[0], pre[1], pre[2], pre[3]};
      set_nibble(np, d, (uint32_t)c);
      if (!it[c].list) {
        push(np, d + 1, d + 1, e + it[c].off, 32, true, nullptr, 0);
      } else {
        const uint32_t st = c ? it[c - 1].next : top.off;
        push(np, d + 1, d + 1, e + st, it[c].next - st, false, nullptr, 0);
      }
      mask |= 1u << c;
    }
    const uint64_t r = rbase + atomicAdd(rcount, 1ULL);
    for (int q = 0; q < 4; ++q) {
      R.rk[4 * r + q] = pre[q];
      R.rbref[4 * r + q] = own[q];
      R.rref[4 * r + q] = I.pref[4 * i + q];
    }
    R.rt[r] = trie;
    R.rd[r] = (uint8_t)a;
    R.rdb[r] = (uint8_t)d;
    R.rvo[r] = 0;
    R.rvl[r] = 0;
    R.rbrl[r] = (uint8_t)ownl;
    R.rrl[r] = I.prl[i];
    R.rmask[r] = (uint16_t)mask;
    R.rlive[r] = REC_LIVE;
    return;
  }
  if (k != 2 || it[0].list || it[0].len == 0 || d != a) return bad(OPEN_BAD);  // a leaf / extension hangs where it starts
  uint8_t nib[64];
  uint32_t np = 0;
  bool leaf = false;
  hp_nibbles(e + it[0].off, it[0].len, &np, &leaf, nib);
  uint64_t key[4] = {pre[0], pre[1], pre[2], pre[3]};
  if (d + np > 64) return bad(OPEN_BAD);
  for (uint32_t q = 0; q < np; ++q) set_nibble(key, d + q, nib[q]);
  if (leaf) {  // [HP(path, leaf), value]: the key is complete (32-byte keys)
    if (d + np != 64 || it[1].list) return bad(OPEN_BAD);
    const uint64_t vo = atomicAdd(heap_n, (unsigned long long)it[1].len);
    for (uint32_t q = 0; q < it[1].len; ++q) heap[vo + q] = e[it[1].off + q];
    const uint64_t r = rbase + atomicAdd(rcount, 1ULL);
    for (int q = 0; q < 4; ++q) {
      R.rk[4 * r + q] = key[q];
      R.rbref[4 * r + q] = 0;
      R.rref[4 * r + q] = I.pref[4 * i + q];
    }
    R.rt[r] = trie;
    R.rd[r] = (uint8_t)a;
    R.rdb[r] = EL_LEAF;
    R.rvo[r] = vo;
    R.rvl[r] = it[1].len;
    R.rbrl[r] = 0;
    R.rrl[r] = I.prl[i];
    R.rmask[r] = 0;
    R.rlive[r] = REC_LIVE;
    atomicAdd(leaves, 1ULL);
    return;
  }
  // extension [HP(shared, ext), ref]: its branch child gets the extension's record (anchor a)
  if (np == 0) return bad(OPEN_BAD);
  if (!it[1].list) {
    if (it[1].len != 32) return bad(OPEN_BAD);
    push(key, a, d + np, e + it[1].off, 32, true, I.pref + 4 * i, I.prl[i]);
  } else {
    push(key, a, d + np, e + it[0].next, it[1].next - it[0].next, false, I.pref + 4 * i, I.prl[i]);
  }
}

struct FCommit {  // one commit's inputs (device buffers)
  const uint32_t* up_trie = nullptr;  // nullable: trie 0
  const uint8_t* up_keys = nullptr;
  const uint8_t* up_vals = nullptr;
  const uint64_t* up_voff = nullptr;
  uint64_t nup = 0;
  const uint32_t* del_trie = nullptr;
  const uint8_t* del_keys = nullptr;
  uint64_t ndel = 0;
  uint32_t klen = 32;
  // an error word of earlier stream work (kh_block_commit's injection) checked at the sort's
  // sync, before the commit changes anything: equal to chk_tok -> KH_EINVAL chk_msg
  const unsigned long long* chk = nullptr;
  unsigned long long chk_tok = 0;
  const char* chk_msg = nullptr;
  // deferred values (kh_block_commit's account phase, run beside the storage phase): the
  // key-only work -- hashing, sort, descent, gather -- is enqueued first; before_values (host)
  // returns once vals_ready has been recorded (the storage roots' injection into up_vals), the
  // stream waits on it, and only then are the values copied into the heap and `chk` read (at
  // the gather's sync, still before the commit changes anything)
  std::function<void()> before_values;
  hipEvent_t vals_ready = nullptr;
  // deferred values: the upserts whose bodies the producer changes (late[i] != ~0, by upsert
  // index; kh_block_commit: those naming a storage trie); the rest are copied and their leaves
  // encoded and hashed before before_values (nullable: every value waits)
  const uint32_t* late = nullptr;
  std::function<bool()> late_ready;  // (host) the late values are already on the device
  // the new roots are on the device (d_tries / d_roots, right after the element build; the
  // records and the anchor map still follow): kh_block_commit's storage phase injects them
  // into the account bodies here, so the account phase need not wait for the rest
  std::function<void(hipStream_t, uint32_t)> after_roots;  // (the stream, the commit's trie count)
  hipEvent_t inputs_ready = nullptr;  // the inputs were staged on another stream (HostPack): wait first
};

static int emit_nodes_dev(kh_ctx* c, DevBuf& out, uint64_t* n_nodes, uint64_t* rlp_len);
static void em_append(kh_ctx* c, DevBuf& em, uint64_t& tn, uint64_t& tb, const uint64_t* d_hashes, const uint8_t* src,
                      const std::vector<uint64_t>& list);

// a commit is about to replace the write-back set: the innermost savepoint keeps the set of its
// version (once), and the commit writes into the spare buffer
static void em_save(kh_trie* h) {
  if (h->sps.empty()) return;
  Savepoint& sp = *h->sps.back();
  if (sp.em_saved) return;
  sp.em_saved = true;
  sp.em_valid = h->em_valid;
  sp.em_n = h->em_n;
  sp.em_bytes = h->em_bytes;
  swap_buf(sp.em, h->em);
  swap_buf(h->em, h->em_spare);
}
// journal room for one more commit: nrec saved records, nmap map-log entries
static JSeg journal_reserve(kh_trie* h, uint64_t nrec, uint64_t nmap) {
  hipStream_t st = h->c->st;
  JSeg s;
  s.rpos = h->jrec_n;
  s.rn = nrec;
  const uint64_t rneed = h->jrec_n + nrec + 16, mneed = h->jmap_n + nmap + 16;
  regrow(h->jidx, h->jrec_n * 4, (rneed + rneed / 2) * 4, st);
  regrow(h->jrec, h->jrec_n * REC_BYTES, (rneed + rneed / 2) * REC_BYTES, st);
  regrow(h->jmap, h->jmap_n * 24, (mneed + mneed / 2) * 24, st);
  return s;
}

// One commit of a block's ops into the forest: upserts then deletes, the last op on a
// key winning; deleting an absent key is a no-op.  Fills h->tries / h->roots.  A refused
// batch (KH_EINVAL) leaves the handle as it was, its last roots and write-back set included;
// with a savepoint open (h->sps) every change is journaled for kh_trie_rollback.
static void forest_commit(kh_trie* h, const FCommit& F, kh_stats* stats) {
  kh_ctx* c = h->c;
  hipStream_t st = c->st;
  if (F.inputs_ready) HIPCHK(hipStreamWaitEvent(st, F.inputs_ready, 0));
  if (stats) memset(stats, 0, sizeof(*stats));
  const bool journal = !h->sps.empty();
  const uint64_t nops = F.nup + F.ndel;
  if (nops == 0) {
    em_save(h);
    h->tries.clear();
    h->roots.clear();
    h->em_valid = false;
    return;
  }
  if (nops >= (1ULL << 30)) throw KhError{KH_EINVAL, "batch too large"};
  if (!(h->flags & KH_HASH_KEYS) && F.klen != 32) throw KhError{KH_EINVAL, "keys must be 32 bytes unless KH_HASH_KEYS"};
  if (F.klen == 0 || F.klen > 4096) throw KhError{KH_EINVAL, "bad key length"};
  // the previous commit's in-flight tail (records, anchor map): its flags before this
  // commit's descent reads the map (done by now, stream order; a failure refuses the handle)
  trie_settle(h);
  HIPCHK(hipEventRecord(c->ev[6], st));
  // ---- 1. op keys (the trie's key encoder), trie ids, sort by (trie, key), last op wins
  const bool segd = h->forest;
  std::vector<size_t> sz = {nops * 32, nops * 4, nops * 8, nops * 8, nops * 4, nops * 4, nops * 32, nops * 4,
                            radix_scratch_bytes(nops), scan_scratch_bytes(nops + 1, 8), CTR_N * 8,
                            nops, nops * 4, nops * 4, nops * 4, (nops + 1) * 8, nops * 8, nops * 4};
  h->ws.ensure(carve_size(sz));
  Carver cv{(char*)h->ws.p, 0, h->ws.cap};
  uint64_t* K = cv.take<uint64_t>(nops * 4);
  uint32_t* Tid = cv.take<uint32_t>(nops);
  SortIO S{};
  S.K32 = K;
  S.n = nops;
  S.ck0 = cv.take<uint64_t>(nops);
  S.ck1 = cv.take<uint64_t>(nops);
  S.idx0 = cv.take<uint32_t>(nops);
  S.idx1 = cv.take<uint32_t>(nops);
  S.skey = cv.take<uint64_t>(nops * 4);
  uint32_t* sseg = cv.take<uint32_t>(nops);
  S.sseg = segd ? sseg : nullptr;
  S.seg = segd ? Tid : nullptr;
  // the trie ids' bits: a hint from the ids committed before (two bits of headroom; the sort is
  // redone with 32 if an id needs more), so the sorted 32-bit prefix holds key bits too and
  // runs of equal prefixes (one per trie with all 32) stay short
  S.sb = segd ? (h->tid_bits ? std::max(h->tid_bits, 1u) : 32u) : 0;
  // keccak'd keys, a few ops per trie: the leading 24 composite bits (the tie kernel orders the
  // rare runs past them; 2^17 ops over the 2^(sb - 2) tries the hint allows, 2^19 in one trie)
  // That assumes keys spread evenly over the tries: one hot trie with thousands of slot writes
  // makes runs past the tie kernel, and the whole sort falls back to 256 bits.  Such a fallback
  // turns the 24-bit form off for the handle's next 16 commits.  Unhashed keys (structured, their
  // leading bytes often equal) never take it.
  if ((h->flags & KH_HASH_KEYS) && S.sb <= 18 && nops <= (segd ? (1ull << 17) : (1ull << 19)) && h->lo24_off == 0)
    S.rs_lo = 40;
  if (h->lo24_off) --h->lo24_off;
  S.rs_scratch = cv.take<char>(radix_scratch_bytes(nops));
  S.scan_scratch = cv.take<char>(scan_scratch_bytes(nops + 1, 8));
  S.ctr = cv.take<unsigned long long>(CTR_N);
  const bool defer = (bool)F.before_values;
  S.chk = defer ? nullptr : F.chk;
  uint8_t* kind = cv.take<uint8_t>(nops);
  uint32_t* tflag = cv.take<uint32_t>(nops);
  uint32_t* tpos = cv.take<uint32_t>(nops);
  uint32_t* isup = cv.take<uint32_t>(nops);
  uint64_t* uoff = cv.take<uint64_t>(nops + 1);
  uint64_t* ulen = cv.take<uint64_t>(nops);
  uint32_t* ur = cv.take<uint32_t>(nops);
  if (segd && ((F.nup && !F.up_trie) || (F.ndel && !F.del_trie))) throw KhError{KH_EINVAL, "forest ops need trie ids"};
  // the op keys (unless hashed above) and trie ids, upserts then deletes: one launch
  bool copy_keys = !(h->flags & KH_HASH_KEYS);
  if (copy_keys && (((uintptr_t)F.up_keys | (uintptr_t)F.del_keys) & 7)) {  // unaligned caller keys: copies
    if (F.nup) HIPCHK(hipMemcpyAsync(K, F.up_keys, F.nup * 32, hipMemcpyDeviceToDevice, st));
    if (F.ndel) HIPCHK(hipMemcpyAsync(K + 4 * F.nup, F.del_keys, F.ndel * 32, hipMemcpyDeviceToDevice, st));
    copy_keys = false;
  }
  // (also zeroes the sort's counters S.ctr)
  hipLaunchKernelGGL(k_f_inputs, GRID(nops, BS), dim3(BS), 0, st, (const uint64_t*)F.up_keys, F.nup,
                     (const uint64_t*)F.del_keys, F.ndel, copy_keys, segd ? F.up_trie : nullptr,
                     segd ? F.del_trie : nullptr, K, Tid, S.ctr);
  // the keys hashed (the trie's key encoder) and the composite sort keys made, one launch
  {
    const bool hk = h->flags & KH_HASH_KEYS;
    const uint32_t* sg = segd ? Tid : nullptr;
    unsigned long long* fl = S.ctr + CTR_TIE;
    uint32_t* hdr = (uint32_t*)S.rs_scratch;
    if (hk && F.klen <= 135)
      hipLaunchKernelGGL((k_f_keys_ck<true, true>), GRID(nops, BS), dim3(BS), 0, st, F.up_keys, F.nup, F.del_keys, F.ndel,
                         F.klen, K, sg, S.sb, S.ck0, S.idx0, fl, hdr);
    else if (hk)
      hipLaunchKernelGGL((k_f_keys_ck<false, true>), GRID(nops, BS), dim3(BS), 0, st, F.up_keys, F.nup, F.del_keys,
                         F.ndel, F.klen, K, sg, S.sb, S.ck0, S.idx0, fl, hdr);
    else
      hipLaunchKernelGGL((k_f_keys_ck<true, false>), GRID(nops, BS), dim3(BS), 0, st, F.up_keys, F.nup, F.del_keys,
                         F.ndel, F.klen, K, sg, S.sb, S.ck0, S.idx0, fl, hdr);
  }
  LAUNCH_CHECK();
  S.ck_made = true;
  sort_dedup(c, S);
  if (S.fallback && S.rs_lo == 40) h->lo24_off = 16;
  if (!defer && F.chk && c->h_pinned[1] == F.chk_tok) throw KhError{KH_EINVAL, F.chk_msg};
  const uint64_t nd = S.m;
  uint32_t* otrie = segd ? S.sseg : sseg;  // the compaction of duplicates moves the sorted ids
  // the descent's touched list and the commit's flags (fctr, zeroed by k_f_prep): [0] touched
  // count, [1] replaced leaves, [2] anchor-map error, [3] refusal / map insert error,
  // [4] fresh map slots, [5] element count, [6] value-only branches made, [7] the hashed ones
  h->tlb.ensure(carve_size({nd * 70 * 4 + 64, 64, nd + 64}));
  Carver c3{(char*)h->tlb.p, 0, h->tlb.cap};
  uint32_t* tlist = c3.take<uint32_t>(nd * 70 + 16);
  unsigned long long* fctr = c3.take<unsigned long long>(8);
  uint8_t* vbf = c3.take<uint8_t>(nd + 64);  // ops that make a value-only branch
  // kinds, the distinct tries of the batch (sorted: the segments of the element build), and
  // the upserts' ranks and value offsets (their values go to the heap)
  hipLaunchKernelGGL(k_f_prep, GRID(nd, BS), dim3(BS), 0, st, (const uint32_t*)S.sidx, nd, F.nup, segd, otrie,
                     F.up_voff, kind, tflag, isup, ulen, fctr);
  LAUNCH_CHECK();
  FOps O{(const uint64_t*)S.skey, (const uint32_t*)otrie, (const uint8_t*)kind, nd};
  uint32_t* ntp = (uint32_t*)(S.ctr + 12);
  uint32_t* nupp = (uint32_t*)(S.ctr + 13);
  if (nd <= SCAN_SMALL_MAX) {  // the three scans in one launch
    hipLaunchKernelGGL(k_scan_small3, dim3(3), dim3(SCAN_SMALL_THREADS), 0, st, ScanJob{tflag, tpos, ntp, false},
                       ScanJob{isup, ur, nupp, false}, ScanJob{ulen, uoff, S.ctr + 14, true}, nd);
    LAUNCH_CHECK();
  } else {
    scan_exclusive<uint32_t>(tflag, tpos, nd, ntp, S.scan_scratch, st);
    scan_exclusive<uint32_t>(isup, ur, nd, nupp, S.scan_scratch, st);
    scan_exclusive<uint64_t>(ulen, uoff, nd, (uint64_t*)(S.ctr + 14), S.scan_scratch, st);
  }
  HIPCHK(hipMemcpyAsync(c->h_pinned, S.ctr + 12, 3 * 8, hipMemcpyDeviceToHost, st));
  HIPCHK(hipStreamSynchronize(st));
  const uint32_t nt = (uint32_t)c->h_pinned[0], nups = (uint32_t)c->h_pinned[1];
  const uint64_t ubytes = c->h_pinned[2];
  // ---- trie list; upsert values into the heap (appended past heap_n, which moves only once
  // the commit is accepted): uoff is the exclusive scan of their lengths over the sorted
  // ops, uo the same offsets by upsert rank (uo[nups] = total)
  h->tbuf.ensure(carve_size({(uint64_t)nt * 4, (uint64_t)nt * 32, 64}));
  Carver ct{(char*)h->tbuf.p, 0, h->tbuf.cap};
  uint32_t* tries = ct.take<uint32_t>(nt);
  uint64_t* roots = ct.take<uint64_t>((uint64_t)nt * 4);
  unsigned long long* tail = ct.take<unsigned long long>(8);  // k_f_roots: the final flags
  h->d_tries = tries;
  h->d_roots = roots;
  regrow(h->heap, h->heap_n, h->heap_n + ubytes + 64, st);
  const uint64_t hb = h->heap_n;
  h->ubuf.ensure(((uint64_t)nups + 1) * 8 + 64);
  uint64_t* uo = (uint64_t*)h->ubuf.p;
  // ---- the elements' buffer: upserts (values in the heap), untouched children, kept
  // leaves, roots.  Sized from the last commit's touched count (or 4 per op) so the descent
  // and the gather need no host round trip between them; a short buffer is grown to the
  // exact size and gathered again after the one sync below.  (Touched records are live
  // records: at most rn - rdead; a guess past 1M touched records -- 16M elements -- is left
  // to the exact second pass.)
  const uint64_t tl_cap = nd * 70 + 16;
  uint64_t ntl_guess = std::max<uint64_t>(4 * nd, h->ntl_hint + h->ntl_hint / 4);
  ntl_guess = std::min({ntl_guess, tl_cap, h->rn - h->rdead + 16, (uint64_t)1 << 20});
  Elems E{};
  auto carve_elems = [&](uint64_t ntl_cap) {
    const uint64_t ecap = (uint64_t)nups + 16 * ntl_cap + nt + 16;
    h->ebuf.ensure(
        carve_size({ecap * 32, ecap * 4, ecap, ecap * 32, ecap, ecap * 8, ecap * 4, ecap * 4, ecap, ecap * 32, ecap, ecap, 64}));
    Carver ce{(char*)h->ebuf.p, 0, h->ebuf.cap};
    E = Elems{};
    E.key = ce.take<uint64_t>(ecap * 4);
    E.seg = ce.take<uint32_t>(ecap);
    E.db = ce.take<uint8_t>(ecap);
    E.bref = ce.take<uint64_t>(ecap * 4);
    E.brl = ce.take<uint8_t>(ecap);
    E.vo = ce.take<uint64_t>(ecap);
    E.vl = ce.take<uint32_t>(ecap);
    E.src = ce.take<uint32_t>(ecap);
    E.oldd = ce.take<uint8_t>(ecap);
    E.cref = ce.take<uint64_t>(ecap * 4);
    E.crl = ce.take<uint8_t>(ecap);
    E.late = ce.take<uint8_t>(ecap);
    E.n = fctr + 5;
    E.cap = ecap;
    return ecap;
  };
  uint64_t ecap = carve_elems(ntl_guess);
  hipLaunchKernelGGL(k_f_ops_post, GRID(nd * CG, BS), dim3(BS), 0, st, O, (const uint32_t*)S.sidx, (const uint32_t*)ur,
                     F.up_vals, F.up_voff, (const uint64_t*)uoff, uo, (uint64_t)nups, ubytes, (uint8_t*)h->heap.p, hb,
                     (const uint32_t*)tflag, (const uint32_t*)tpos, tries, E, true, !defer ? 1 : F.late ? 2 : 0,
                     F.late);
  LAUNCH_CHECK();
  // ---- 2. descent: opened branches and touched leaves
  recs_reserve(h, h->rn + 16);
  if (h->mcap == 0) map_rebuild(h, nops + 1024);
  h->flags_dirty = true;  // until the touched records die (k_map_delete) or are untouched
  hipLaunchKernelGGL(k_f_descend, GRID(nd, BS), dim3(BS), 0, st, O, map_of(h), recs_of(h), (uint32_t*)h->touched.p,
                     (uint8_t*)h->replaced.p, tlist, fctr, vbf);
  LAUNCH_CHECK();
  // ---- 3. elements: the gather (grid-stride over the device's touched count), one sync
  auto gather = [&](bool redo) {
    if (redo)  // the upserts' elements again, into the grown buffer
      hipLaunchKernelGGL(k_f_upsert_elems, GRID(nd, BS), dim3(BS), 0, st, O, (const uint32_t*)tries, nt,
                         (const uint32_t*)ur, (const uint64_t*)uo, E, hb, (uint64_t)nups, (const uint32_t*)S.sidx,
                         F.late);
    const uint64_t gblocks = std::min<uint64_t>((uint64_t)c->n_cu * KH_GATHER_PER_CU, (nd * 16 * 8 + GATHER_BS - 1) / GATHER_BS);
    hipLaunchKernelGGL(k_f_gather, dim3((unsigned)std::max<uint64_t>(gblocks, 1)), dim3(GATHER_BS), 0, st, map_of(h),
                       recs_of(h), (const uint32_t*)h->touched.p, (const uint8_t*)h->replaced.p,
                       (const uint32_t*)tlist, (const unsigned long long*)fctr, (const uint32_t*)tries, nt, E, fctr);
    LAUNCH_CHECK();
    HIPCHK(hipMemcpyAsync(c->h_pinned, fctr, 56, hipMemcpyDeviceToHost, st));  // [0..6]
    HIPCHK(hipStreamSynchronize(st));
  };
  gather(false);
  const uint64_t ntl = c->h_pinned[0], nrep = c->h_pinned[1];
  if (c->h_pinned[2] == 3) throw KhError{KH_EINTERNAL, "forest descent: corrupt anchor map"};
  if (c->h_pinned[3]) {  // nothing has changed yet: clear the descent's flags and refuse the batch
    if (ntl) {
      hipLaunchKernelGGL(k_f_untouch, GRID(ntl, BS), dim3(BS), 0, st, (const uint32_t*)tlist, ntl,
                         (uint32_t*)h->touched.p, (uint8_t*)h->replaced.p);
      LAUNCH_CHECK();
      HIPCHK(hipStreamSynchronize(st));
    }
    h->flags_dirty = false;
    throw KhError{KH_EINVAL,
                  "remove of a key held by a value-only branch: khipu's fix of the emptied branch throws "
                  "MPTException(\"Branch with no subvalues\") (MerklePatriciaTrie.scala:323-370,430-477); the trie "
                  "is unchanged"};
  }
  if (c->h_pinned[2]) throw KhError{KH_EINTERNAL, "forest gather: corrupt anchor map"};
  uint64_t ne = c->h_pinned[5];
  if (ne > ecap) {  // the guess was short: the exact capacity, gathered again
    ecap = carve_elems(ntl);
    gather(true);
    ne = c->h_pinned[5];
    if (c->h_pinned[2]) throw KhError{KH_EINTERNAL, "forest gather: corrupt anchor map"};
  }
  if (ne > ecap) throw KhError{KH_EINTERNAL, "forest gather: element overflow"};
  // deferred values: once their producer is done (the host waits for its event to be recorded,
  // the stream for the event), the values into the heap -- right before the element build's
  // leaves read them, so the element sort and topology run beside the producer too
  bool values_in = !defer;
  auto values_now = [&] {
    if (values_in) return;
    values_in = true;
    F.before_values();
    if (F.vals_ready) HIPCHK(hipStreamWaitEvent(st, F.vals_ready, 0));
    hipLaunchKernelGGL(k_f_ops_post, GRID(nd * CG, BS), dim3(BS), 0, st, O, (const uint32_t*)S.sidx,
                       (const uint32_t*)ur, F.up_vals, F.up_voff, (const uint64_t*)uoff, uo, (uint64_t)nups, ubytes,
                       (uint8_t*)h->heap.p, hb, (const uint32_t*)tflag, (const uint32_t*)tpos, tries, E, false,
                       F.late ? 3 : 1, F.late);
    LAUNCH_CHECK();
  };
  // value-only branches (rare: a re-put of a key sharing 63 nibbles with another): their
  // encodings need the values, so a deferred producer is waited for here
  const uint64_t nvb = c->h_pinned[6];
  std::vector<uint64_t> vb_list;  // (encoding offset, length) of the hashed ones
  DevBuf vbenc;
  uint64_t* vbh = nullptr;
  if (nvb) {
    values_now();
    vbenc.ensure(ubytes + 32 * (uint64_t)nups + 64 + nvb * 48 + 64);
    uint8_t* enc = (uint8_t*)vbenc.p;
    uint64_t* vbl = (uint64_t*)(enc + ((ubytes + 32 * (uint64_t)nups + 64 + 15) & ~(uint64_t)15));
    vbh = vbl + 2 * nvb;
    unsigned long long* vcnt = fctr + 7;
    hipLaunchKernelGGL(k_f_vb_elems, GRID(nd, BS), dim3(BS), 0, st, O, (const uint8_t*)vbf, (const uint32_t*)ur,
                       (const uint64_t*)uoff, (const uint8_t*)h->heap.p, E, enc, vbl, vbh, vcnt);
    LAUNCH_CHECK();
    if (h->flags & KH_EMIT_NODES) {
      HIPCHK(hipMemcpyAsync(c->h_pinned, vcnt, 8, hipMemcpyDeviceToHost, st));
      HIPCHK(hipStreamSynchronize(st));
      const uint64_t nh = c->h_pinned[0];
      vb_list.resize(2 * nh);
      if (nh) HIPCHK(hipMemcpy(vb_list.data(), vbl, 16 * nh, hipMemcpyDeviceToHost));
    }
  }
  h->ntl_hint = ntl;
  h->heap_n = hb + ubytes;
  HIPCHK(hipEventRecord(c->ev[7], st));
  // ---- 4. element build (every touched trie a segment), or all tries emptied
  BuildOut O2;
  kh_stats bst{};
  uint64_t B = 0, m = 0;
  const bool keep_em = h->flags & KH_EMIT_NODES;
  if (ne) {
    ElemArgs EA{E.db, E.bref, E.brl, E.oldd, E.cref, E.crl, (defer && F.late) ? E.late : nullptr, &h->elout, &h->eloutb};
    // encodings are kept (emit path) only when the handle hands out its write-back set;
    // otherwise the fused branch levels (one launch per level, no message arena)
    BuildArgs A{(const uint8_t*)E.key, 32, (const uint8_t*)h->heap.p, (const uint64_t*)E.vo, ne,
                nt > 1 ? (const uint32_t*)E.seg : nullptr, nt, 0, 0, keep_em};
    A.vlen = E.vl;
    A.el = &EA;
    A.dev_results = true;  // the counters come back with the roots (build_stats below)
    if (defer) A.before_leaves = values_now;
    if (defer) A.late_ready = F.late_ready;
    run_build(c, A, O2, &bst);
    B = c->last_B;
    m = c->T.m;
    if (m != ne) throw KhError{KH_EINTERNAL, "forest: duplicate elements"};
  }
  // Without a write-back set or a map rebuild, the commit returns as soon as its roots are on
  // the host; the records and the anchor map follow on the stream (the next call is ordered
  // after them, trie_settle reads their flags): configs[2]'s account phase ends 0.1 ms sooner
  const bool rebuild = ne && 2 * (h->mused + B + m + 1024) > h->mcap;
  const bool lazy = ne && !keep_em && !rebuild;
  const size_t o_roots = (size_t)((char*)roots - (char*)tries), o_tail = (size_t)((char*)tail - (char*)tries);
  uint8_t* hs = nullptr;
  if (ne && (lazy || F.after_roots)) {  // the roots now (k_f_roots runs again with the final flags below)
    hipLaunchKernelGGL(k_f_roots, GRID(nt, BS), dim3(BS), 0, st, (const uint64_t*)c->T.res_hash,
                       (const uint32_t*)c->T.res_len, nt, roots, (const unsigned long long*)c->T.ctr,
                       (const unsigned long long*)fctr, tail);
    LAUNCH_CHECK();
    if (F.after_roots) F.after_roots(st, nt);
    if (lazy) {
      if (!h->ev_roots) HIPCHK(hipEventCreateWithFlags(&h->ev_roots, hipEventDisableTiming));
      if (!h->pend_ev) HIPCHK(hipEventCreateWithFlags(&h->pend_ev, hipEventDisableTiming));
      if (!h->pend) HIPCHK(hipHostMalloc((void**)&h->pend, 64, hipHostMallocDefault));
      hs = pinned_stage(c, o_tail + 64);
      HIPCHK(hipMemcpyAsync(hs, tries, o_tail + 64, hipMemcpyDeviceToHost, st));
      if (defer && F.chk) HIPCHK(hipMemcpyAsync(c->h_pinned + 8, F.chk, 8, hipMemcpyDeviceToHost, st));
      HIPCHK(hipEventRecord(h->ev_roots, st));
    }
  }
  values_now();  // (no element build: the producer still finishes before the commit does)
  // ---- 5. records: new branches, re-anchored / new elements; the anchor map follows
  const uint64_t nnew = nups;  // every upsert is a new leaf record
  recs_reserve(h, h->rn + B + nnew + 16);
  const uint64_t base_b = h->rn, base_e = h->rn + B;
  Recs R = recs_of(h);
  AMap M = map_of(h);
  bool count_fresh = false;  // fctr[4] holds this commit's fresh map slots
  uint32_t *isnew = nullptr, *nrank = nullptr, *eid = nullptr, *esrc = nullptr;
  uint8_t* sel = nullptr;
  // journal (a savepoint is open): the records rewritten in place -- the touched ones and the
  // element sources -- saved before the first change; the map deletes' and inserts' slot logs.
  // The segment is listed before the first change, so a failure past it still rolls back.
  uint64_t *dlog = nullptr, *ilog = nullptr;
  auto journal_begin = [&](uint64_t ndel_log, uint64_t nins_log) {
    if (!journal) return;
    JSeg js = journal_reserve(h, ntl + m, ndel_log + nins_log);
    js.dpos = h->jmap_n;
    js.dn = ndel_log;
    js.ipos = js.dpos + ndel_log;
    js.in = 0;  // set once the inserts are launched
    // (the records rewritten in place: the touched ones and the element sources that move --
    // k_f_elem_recs leaves every other source record as it is)
    const uint64_t nsave = ntl + m;
    if (nsave)
      hipLaunchKernelGGL(k_rec_save, GRID(nsave * 8, BS), dim3(BS), 0, st, (const uint8_t*)h->recs.p,
                         (const uint32_t*)tlist, ntl, (const uint32_t*)esrc, m, (uint32_t*)h->jidx.p + js.rpos,
                         (uint8_t*)h->jrec.p + js.rpos * REC_BYTES);
    LAUNCH_CHECK();
    dlog = (uint64_t*)h->jmap.p + 3 * js.dpos;
    ilog = (uint64_t*)h->jmap.p + 3 * js.ipos;
    h->jsegs.push_back(js);
    h->jrec_n += nsave;
    h->jmap_n += ndel_log + nins_log;
  };
  if (ne) {
    h->selb.ensure(carve_size({m + 2 * B, m * 4, m * 4, m * 4, m * 4, m, scan_scratch_bytes(m + 1, 4), 64}));
    Carver cs{(char*)h->selb.p, 0, h->selb.cap};
    sel = cs.take<uint8_t>(m + 2 * B);
    uint8_t* rein = cs.take<uint8_t>(m);
    isnew = cs.take<uint32_t>(m);
    nrank = cs.take<uint32_t>(m);
    eid = cs.take<uint32_t>(m);
    esrc = cs.take<uint32_t>(m);
    void* sscr = cs.take<char>(scan_scratch_bytes(m + 1, 4));
    uint32_t* tot = cs.take<uint32_t>(8);
    Topo T = c->T;
    if (B)
      hipLaunchKernelGGL(k_f_branch_recs, GRID(B, BS), dim3(BS), 0, st, T, (const uint32_t*)(T.ctr + CTR_B),
                         (const uint32_t*)tries, M, R, base_b, sel);
    LAUNCH_CHECK();
    hipLaunchKernelGGL(k_f_elem_flags, GRID(m, BS), dim3(BS), 0, st, T, E, (const uint32_t*)h->touched.p, sel, isnew,
                       esrc, rein);
    LAUNCH_CHECK();
    scan_exclusive<uint32_t>(isnew, nrank, m, tot, sscr, st);
    journal_begin(ntl + m, B + m);
    // old anchors out of the map (touched records, element sources), then touched records die
    hipLaunchKernelGGL(k_map_delete, GRID(ntl + m, BS), dim3(BS), 0, st, M, R, (const uint32_t*)tlist, ntl,
                       (const uint32_t*)esrc, m, (uint32_t*)h->touched.p, (uint8_t*)h->replaced.p, dlog);
    LAUNCH_CHECK();
    h->flags_dirty = false;
    hipLaunchKernelGGL(k_f_elem_recs, GRID(m, BS), dim3(BS), 0, st, T, E, (const uint32_t*)tries,
                       (const uint32_t*)nrank, (const uint8_t*)rein, R, base_e, eid);
    LAUNCH_CHECK();
    // map capacity: rebuild when live + tombstones would pass half the table
    h->rn = base_e + nnew;
    if (rebuild) {
      map_rebuild(h, B + m);
    } else {
      // (the table's load grows by the inserts that took an empty slot: fctr[4], read at the
      // final sync; B + m bounds it for the rebuild test above)
      hipLaunchKernelGGL(k_map_insert, GRID(B + m, BS), dim3(BS), 0, st, M, R, base_b, B, (const uint32_t*)eid, m,
                         fctr + 3, fctr + 4, ilog);
      LAUNCH_CHECK();
      if (ilog) h->jsegs.back().in = B + m;
      count_fresh = true;
    }
    if (lazy) {  // the map's flags to the handle's pinned word pair, read by trie_settle
      HIPCHK(hipMemcpyAsync(h->pend, fctr + 3, 16, hipMemcpyDeviceToHost, st));
      HIPCHK(hipEventRecord(h->pend_ev, st));
      h->pend_valid = true;
      h->pend_fresh = count_fresh;
    } else {
      hipLaunchKernelGGL(k_f_roots, GRID(nt, BS), dim3(BS), 0, st, (const uint64_t*)T.res_hash,
                         (const uint32_t*)T.res_len, nt, roots, (const unsigned long long*)T.ctr,
                         (const unsigned long long*)fctr, tail);
      LAUNCH_CHECK();
    }
  } else {
    journal_begin(ntl, 0);
    if (ntl)
      hipLaunchKernelGGL(k_map_delete, GRID(ntl, BS), dim3(BS), 0, st, M, R, (const uint32_t*)tlist, ntl,
                         (const uint32_t*)nullptr, (uint64_t)0, (uint32_t*)h->touched.p, (uint8_t*)h->replaced.p,
                         dlog);
    h->flags_dirty = false;
    hipLaunchKernelGGL(k_f_roots, GRID(nt, BS), dim3(BS), 0, st, (const uint64_t*)nullptr, (const uint32_t*)nullptr,
                       nt, roots, (const unsigned long long*)nullptr, (const unsigned long long*)fctr, tail);
    LAUNCH_CHECK();
  }
  h->rn = base_e + nnew;
  h->nleaves = h->nleaves + nups - nrep;
  // ---- 6. this commit's write-back set (kept on the device for kh_trie_emit_nodes)
  em_save(h);
  if (keep_em && ne) {
    c->T.emit_sel = sel;
    uint64_t en = 0, eb2 = 0;
    emit_nodes_dev(c, h->em, &en, &eb2);
    c->T.emit_sel = nullptr;
    if (!vb_list.empty()) em_append(c, h->em, en, eb2, vbh, (const uint8_t*)vbenc.p, vb_list);
    h->em_n = en;
    h->em_bytes = eb2;
    h->em_valid = true;
  } else if (keep_em) {
    h->em_n = h->em_bytes = 0;
    h->em_valid = true;
  }
  // ---- roots to the host
  // (through the pinned staging: a pageable destination pins its pages on every copy)
  // One sync: the trie list and roots (carved back to back), the element build's counters
  // and the map's error flag.
  h->tries.resize(nt);
  h->roots.resize((uint64_t)nt * 32);
  // (k_f_roots left the final flags in the tail after the roots: one copy)
  if (lazy) {
    HIPCHK(hipEventSynchronize(h->ev_roots));
  } else {
    hs = pinned_stage(c, o_tail + 64);
    HIPCHK(hipMemcpyAsync(hs, tries, o_tail + 64, hipMemcpyDeviceToHost, st));
    if (defer && F.chk) HIPCHK(hipMemcpyAsync(c->h_pinned + 8, F.chk, 8, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
  }
  // a deferred producer's error word, read at the last sync: the commit has changed the handle
  // by now, so the caller's savepoint takes it back (kh_block_commit always holds one)
  if (defer && F.chk && c->h_pinned[8] == F.chk_tok) throw KhError{KH_EINVAL, F.chk_msg};
  const unsigned long long* ht = (const unsigned long long*)(hs + o_tail);
  if (!lazy && count_fresh) h->mused += ht[6];
  memcpy(h->tries.data(), hs, (uint64_t)nt * 4);
  memcpy(h->roots.data(), hs + o_roots, (uint64_t)nt * 32);
  if (nt && h->forest)  // (sorted: the last is the largest)
    h->tid_bits = std::max(h->tid_bits, std::min(bits_for((uint64_t)h->tries[nt - 1] + 1) + 2, 32u));
  if (ne) build_stats_sums(c, ht, &bst);
  if (!lazy && ht[5]) throw KhError{KH_EINTERNAL, "anchor map insert failed"};
  if (!h->forest) memcpy(h->root, nt ? h->roots.data() : h->root, 32);
  float merge_ms = ev_ms(c->ev[6], c->ev[7]);
  if (stats) {
    *stats = bst;
    stats->n_inputs = nops;
    stats->n_leaves = h->nleaves;
    stats->t_sort_ms = merge_ms;  // batch sort + descent + element gather
    stats->t_total_ms += merge_ms;
  }
}

// ---- versioned commits: savepoint / rollback / release (see Savepoint)
static void trie_savepoint(kh_trie* h) {
  trie_settle(h);
  auto sp = std::make_unique<Savepoint>();
  sp->rn = h->rn;
  sp->heap_n = h->heap_n;
  sp->nleaves = h->nleaves;
  sp->mused = h->mused;
  sp->rdead = h->rdead;
  sp->map_epoch = h->map_epoch;
  memcpy(sp->root, h->root, 32);
  sp->tries = h->tries;
  sp->roots = h->roots;
  sp->seg0 = h->jsegs.size();
  sp->jrec0 = h->jrec_n;
  sp->jmap0 = h->jmap_n;
  h->sps.push_back(std::move(sp));
}
// back to the innermost savepoint's version: the journaled commits undone newest first (map
// inserts, map deletes, then the records they rewrote), the appended records cut off (and
// cleared), the host-side fields restored; the anchor map is rebuilt instead when it was
// rebuilt (resized) after the savepoint
static void trie_rollback(kh_trie* h) {
  if (h->sps.empty()) throw KhError{KH_EINVAL, "no open savepoint"};
  try {
    trie_settle(h);
  } catch (const KhError&) {  // (the journal undoes that commit's map writes all the same)
  }
  // (a savepoint is opened only on a settled, usable handle: a broken tail came after it)
  hipStream_t st = h->c->st;
  Savepoint& sp = *h->sps.back();
  const bool remap = h->map_epoch != sp.map_epoch;
  if (h->flags_dirty) {  // a commit failed between its descent and its map update
    if (h->rn) {
      HIPCHK(hipMemsetAsync(h->touched.p, 0, h->rn * 4, st));
      HIPCHK(hipMemsetAsync(h->replaced.p, 0, h->rn, st));
    }
    h->flags_dirty = false;
  }
  const AMap M = map_of(h);
  for (size_t k = h->jsegs.size(); k-- > sp.seg0;) {
    const JSeg& s = h->jsegs[k];
    const uint64_t* jm = (const uint64_t*)h->jmap.p;
    if (!remap && s.in) hipLaunchKernelGGL(k_map_undo, GRID(s.in, BS), dim3(BS), 0, st, M, jm + 3 * s.ipos, s.in);
    if (!remap && s.dn) hipLaunchKernelGGL(k_map_undo, GRID(s.dn, BS), dim3(BS), 0, st, M, jm + 3 * s.dpos, s.dn);
    if (s.rn)
      hipLaunchKernelGGL(k_rec_restore, GRID(s.rn * 8, BS), dim3(BS), 0, st, (uint8_t*)h->recs.p,
                         (const uint32_t*)h->jidx.p + s.rpos, (const uint8_t*)h->jrec.p + s.rpos * REC_BYTES, s.rn);
    LAUNCH_CHECK();
  }
  if (h->rn > sp.rn)
    HIPCHK(hipMemsetAsync((uint8_t*)h->recs.p + sp.rn * REC_BYTES, 0, (h->rn - sp.rn) * REC_BYTES, st));
  h->rn = sp.rn;
  h->heap_n = sp.heap_n;
  h->nleaves = sp.nleaves;
  h->mused = sp.mused;
  h->rdead = sp.rdead;
  memcpy(h->root, sp.root, 32);
  h->tries = sp.tries;
  h->roots = sp.roots;
  h->d_tries = nullptr;
  h->d_roots = nullptr;
  h->jsegs.resize(sp.seg0);
  h->jrec_n = sp.jrec0;
  h->jmap_n = sp.jmap0;
  if (sp.em_saved) {
    swap_buf(h->em_spare, h->em);
    swap_buf(h->em, sp.em);
    h->em_valid = sp.em_valid;
    h->em_n = sp.em_n;
    h->em_bytes = sp.em_bytes;
  }
  h->sps.pop_back();
  if (remap) map_rebuild(h, 1024);  // (syncs)
  HIPCHK(hipStreamSynchronize(st));
  h->broken = false;  // back before any failed tail
}
// keep the commits since the innermost savepoint: it is dropped (its saved write-back set
// passes to the enclosing savepoint when that one has none); the journal is emptied when the
// last savepoint goes
static void trie_release(kh_trie* h) {
  if (h->sps.empty()) throw KhError{KH_EINVAL, "no open savepoint"};
  trie_settle(h);  // a commit kept only once its in-flight tail checked out
  std::unique_ptr<Savepoint> sp = std::move(h->sps.back());
  h->sps.pop_back();
  if (!h->sps.empty()) {
    Savepoint& outer = *h->sps.back();
    if (sp->em_saved && !outer.em_saved) {
      outer.em_saved = true;
      outer.em_valid = sp->em_valid;
      outer.em_n = sp->em_n;
      outer.em_bytes = sp->em_bytes;
      swap_buf(outer.em, sp->em);
    }
  } else {
    h->jsegs.clear();
    h->jrec_n = h->jmap_n = 0;
  }
  if (sp->em.p && !h->em_spare.p) swap_buf(h->em_spare, sp->em);
}
// an all-or-nothing section over one or two handles (kh_block_commit, kh_trie_root_of): a
// savepoint on each; rolled back unless released
struct Txn {
  kh_trie* h[2] = {nullptr, nullptr};
  bool open = false;
  Txn(kh_trie* a, kh_trie* b) {
    trie_savepoint(a);
    h[0] = a;
    if (b) {
      try {
        trie_savepoint(b);
      } catch (...) {
        h[0]->sps.pop_back();
        throw;
      }
      h[1] = b;
    }
    open = true;
  }
  void release() {
    for (int i = 1; i >= 0; --i)
      if (h[i]) trie_release(h[i]);
    open = false;
  }
  void rollback() {
    for (int i = 1; i >= 0; --i)
      if (h[i]) trie_rollback(h[i]);
    open = false;
  }
  ~Txn() {
    if (!open) return;
    try {
      rollback();
    } catch (...) {  // a failed rollback leaves the handle as the failure left it (KH_EDEVICE)
    }
  }
};
// MerklePatriciaTrie.copy (MerklePatriciaTrie.scala:556): an independent handle holding the
// current version (records, anchor map, value heap, last roots and write-back set) in HBM
static void make_private(kh_trie* h);
static kh_trie* trie_copy(kh_trie* h) {
  trie_settle(h);
  std::unique_ptr<kh_trie> n(new kh_trie());
  n->c = h->c;
  n->home = h->home;
  n->lk = &h->home->mu;
  n->flags = h->flags;
  n->forest = h->forest;
  hipStream_t st = h->c->st;
  recs_reserve(n.get(), h->rn + 16);
  if (h->rn) HIPCHK(hipMemcpyAsync(n->recs.p, h->recs.p, h->rn * REC_BYTES, hipMemcpyDeviceToDevice, st));
  n->rn = h->rn;
  n->rdead = h->rdead;
  if (h->mcap) {
    n->mslots.ensure(h->mcap * 16);
    HIPCHK(hipMemcpyAsync(n->mslots.p, h->mslots.p, h->mcap * 16, hipMemcpyDeviceToDevice, st));
    n->mcap = h->mcap;
    n->mused = h->mused;
  }
  n->heap.ensure(h->heap_n + 64);
  if (h->heap_n) HIPCHK(hipMemcpyAsync(n->heap.p, h->heap.p, h->heap_n, hipMemcpyDeviceToDevice, st));
  n->heap_n = h->heap_n;
  n->nleaves = h->nleaves;
  memcpy(n->root, h->root, 32);
  n->tries = h->tries;
  n->roots = h->roots;
  n->ntl_hint = h->ntl_hint;
  if (h->em_valid && h->em.p) {
    n->em.ensure(h->em.cap);
    HIPCHK(hipMemcpyAsync(n->em.p, h->em.p, h->em.cap, hipMemcpyDeviceToDevice, st));
  }
  n->em_valid = h->em_valid;
  n->em_n = h->em_n;
  n->em_bytes = h->em_bytes;
  HIPCHK(hipStreamSynchronize(st));
  if (h->priv) make_private(n.get());  // (a copy of a host handle commits beside it too)
  return n.release();
}

// ---- compaction: records and the value heap are append-only between compactions (a commit
// appends the records and values it makes and leaves the ones it replaces dead); trie_compact
// rewrites the live records densely, each with its value moved into a dense heap, and rebuilds
// the anchor map.  Nothing outside the records and the map refers to a record index (roots,
// last roots and the write-back set are hashes and encodings), so the version is unchanged.
__global__ void __launch_bounds__(BS) k_compact_in(Recs R, uint64_t n, uint32_t* live, uint64_t* vlen) {
  const uint64_t i = (uint64_t)blockIdx.x * BS + threadIdx.x;
  if (i >= n) return;
  const bool l = R.rlive[i] == REC_LIVE;
  live[i] = l ? 1u : 0u;
  vlen[i] = l ? R.rvl[i] : 0;
}
// 8 threads per record: one 16-byte quarter-line each, then the value's bytes strided over them
__global__ void __launch_bounds__(BS) k_compact_move(Recs R, uint64_t n, const uint32_t* pos, const uint64_t* hoff,
                                                     const uint8_t* heap, uint8_t* recs2, uint8_t* heap2) {
  const uint64_t t = (uint64_t)blockIdx.x * BS + threadIdx.x, i = t >> 3;
  const uint32_t q = (uint32_t)(t & 7);
  if (i >= n || R.rlive[i] != REC_LIVE) return;
  const uint64_t ho = hoff[i];
  ulonglong2 w = ((const ulonglong2*)(R.rk.b + i * REC_BYTES))[q];
  if (q == 3) w.x = ho;  // rvo: bytes 48..55
  ((ulonglong2*)(recs2 + (uint64_t)pos[i] * REC_BYTES))[q] = w;
  const uint32_t vl = R.rvl[i];
  const uint64_t vo = R.rvo[i];
  for (uint32_t b = q; b < vl; b += 8) heap2[ho + b] = heap[vo + b];
}
static void trie_compact(kh_trie* h, kh_trie_usage_t* before) {
  if (!h->sps.empty()) throw KhError{KH_EINVAL, "kh_trie_compact: a savepoint is open"};
  trie_settle(h);
  kh_ctx* c = h->c;
  hipStream_t st = c->st;
  const uint64_t n = h->rn;
  if (before) {
    before->records = n;
    before->heap_bytes = h->heap_n;
  }
  if (n == 0) return;
  DevBuf wsb;
  const size_t scr = scan_scratch_bytes(n, 8);
  wsb.ensure(n * 4 + n * 8 + scr + 256);
  uint64_t* vlen = (uint64_t*)wsb.p;
  uint32_t* live = (uint32_t*)((char*)wsb.p + n * 8);
  void* scratch = (char*)wsb.p + n * 12 + 64;
  h->merr.ensure(64);
  uint64_t* tot = (uint64_t*)h->merr.p, *tot64 = tot + 1;
  hipLaunchKernelGGL(k_compact_in, GRID(n, BS), dim3(BS), 0, st, recs_of(h), n, live, vlen);
  LAUNCH_CHECK();
  scan_exclusive<uint32_t>(live, live, n, (uint32_t*)tot, scratch, st);
  scan_exclusive<uint64_t>(vlen, vlen, n, tot64, scratch, st);
  HIPCHK(hipMemcpyAsync(c->h_pinned, tot, 16, hipMemcpyDeviceToHost, st));
  HIPCHK(hipStreamSynchronize(st));
  const uint64_t nlive = (uint32_t)c->h_pinned[0], hbytes = c->h_pinned[1];
  const uint64_t cap = std::max<uint64_t>(nlive + nlive / 2, 4096);
  DevBuf recs2, touched2, replaced2, heap2;
  recs2.ensure(cap * REC_BYTES);
  touched2.ensure(cap * 4);
  replaced2.ensure(cap);
  heap2.ensure(hbytes + hbytes / 4 + 64);
  HIPCHK(hipMemsetAsync((uint8_t*)recs2.p + nlive * REC_BYTES, 0, recs2.cap - nlive * REC_BYTES, st));
  HIPCHK(hipMemsetAsync(touched2.p, 0, touched2.cap, st));
  HIPCHK(hipMemsetAsync(replaced2.p, 0, replaced2.cap, st));
  hipLaunchKernelGGL(k_compact_move, GRID(n * 8, BS), dim3(BS), 0, st, recs_of(h), n, (const uint32_t*)live,
                     (const uint64_t*)vlen, (const uint8_t*)h->heap.p, (uint8_t*)recs2.p, (uint8_t*)heap2.p);
  LAUNCH_CHECK();
  HIPCHK(hipStreamSynchronize(st));
  swap_buf(h->recs, recs2);
  swap_buf(h->touched, touched2);
  swap_buf(h->replaced, replaced2);
  swap_buf(h->heap, heap2);
  h->rcap = std::min({h->recs.cap / REC_BYTES, h->touched.cap / 4, h->replaced.cap});
  h->rn = nlive;
  h->heap_n = hbytes;
  h->flags_dirty = false;
  // the per-commit scratch keeps the size of the largest commit so far (the open's build
  // above all): released here, the next commit sizes it again; the write-back set is moved
  // to a buffer of its own size
  for (DevBuf* b : {&h->ws, &h->elout, &h->eloutb, &h->tlb, &h->ebuf, &h->tbuf, &h->ubuf, &h->selb, &h->gbuf,
                    &h->em_spare})
    b->release();
  h->d_tries = nullptr;  // (they lived in tbuf; the block commit's injection uploads them again)
  h->d_roots = nullptr;
  if (h->em.p && h->em_valid && h->em_n) {
    const size_t need = ((h->em_n * 32 + 255) & ~(size_t)255) + ((h->em_bytes + 255) & ~(size_t)255) + (h->em_n + 1) * 8;
    if (need < h->em.cap / 2) {
      DevBuf e2;
      e2.ensure(need);
      HIPCHK(hipMemcpyAsync(e2.p, h->em.p, need, hipMemcpyDeviceToDevice, st));
      HIPCHK(hipStreamSynchronize(st));
      swap_buf(h->em, e2);
    }
  } else {
    h->em.release();
  }
  map_rebuild(h, 1024);  // (syncs; recounts the live records: rdead = 0)
}
static void trie_usage(kh_trie* h, kh_trie_usage_t* u) {
  trie_settle(h);
  kh_ctx* c = h->c;
  hipStream_t st = c->st;
  memset(u, 0, sizeof(*u));
  u->records = h->rn;
  u->heap_bytes = h->heap_n;
  u->map_slots = h->mcap;
  u->hbm_bytes = h->recs.cap + h->touched.cap + h->replaced.cap + h->mslots.cap + h->heap.cap + h->ws.cap +
                 h->elout.cap + h->eloutb.cap + h->em.cap + h->em_spare.cap + h->jidx.cap + h->jrec.cap +
                 h->jmap.cap + h->tlb.cap + h->ebuf.cap + h->tbuf.cap + h->ubuf.cap + h->selb.cap + h->gbuf.cap;
  if (!h->rn) return;
  h->merr.ensure(64);
  unsigned long long* cnt = (unsigned long long*)h->merr.p;
  HIPCHK(hipMemsetAsync(cnt, 0, 16, st));
  hipLaunchKernelGGL(k_rec_count_live, GRID(h->rn, BS), dim3(BS), 0, st, recs_of(h), h->rn, cnt);
  hipLaunchKernelGGL(k_heap_live, GRID(h->rn, BS), dim3(BS), 0, st, recs_of(h), h->rn, cnt + 1);
  LAUNCH_CHECK();
  HIPCHK(hipMemcpyAsync(c->h_pinned, cnt, 16, hipMemcpyDeviceToHost, st));
  HIPCHK(hipStreamSynchronize(st));
  u->live_records = c->h_pinned[0];
  u->live_heap_bytes = c->h_pinned[1];
}

// ---------------------------------------------------------------------------
// C ABI
// ---------------------------------------------------------------------------
extern "C" {

const char* kh_last_error(void) { return g_err.c_str(); }
const char* kh_version(void) { return "khst 0.1 (gfx950)"; }
int kh_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

int kh_ctx_create(int device, kh_ctx** out) { API_TRY(*out = ctx_new(device)) }

int kh_ctx_destroy(kh_ctx* c) {
  if (!c) return KH_OK;
  API_TRY({
    (void)hipSetDevice(c->dev);
    (void)hipStreamSynchronize(c->st);
    if (c->bsub) (void)kh_ctx_destroy(c->bsub);
    if (c->bev) (void)hipEventDestroy(c->bev);
    for (DevBuf* b : {&c->ws_inject, &c->ws_list, &c->ws1, &c->ws2, &c->ws3, &c->in_keys, &c->in_vals, &c->in_voff, &c->in_seg, &c->in_kn, &c->in_aux, &c->in_block, &c->out_emit,
                      &c->emit_dev})
      b->release();
    for (auto& e : c->ev)
      if (e) (void)hipEventDestroy(e);
    if (c->h_pinned) (void)hipHostFree(c->h_pinned);
    if (c->h_res) (void)hipHostFree(c->h_res);
    c->hworker.reset();  // (idle: every call joins its stager before returning)
    if (c->cs) (void)hipStreamSynchronize(c->cs);
    if (c->ring) (void)hipHostFree(c->ring);
    for (auto& e : c->ring_ev)
      if (e) (void)hipEventDestroy(e);
    for (auto e : c->part_ev) (void)hipEventDestroy(e);
    if (c->cs) (void)hipStreamDestroy(c->cs);
    if (c->pack_ev) {
      (void)hipEventSynchronize(c->pack_ev);
      (void)hipEventDestroy(c->pack_ev);
    }
    if (c->h_pack) (void)hipHostFree(c->h_pack);
    if (c->own) (void)hipStreamDestroy(c->own);
    if (c->st2) (void)hipStreamDestroy(c->st2);
    delete c;
  })
}

int kh_ctx_set_stream(kh_ctx* c, void* s) {
  if (!c) return set_err(KH_EINVAL, "null context");
  c->st = s ? (hipStream_t)s : c->own;
  return KH_OK;
}

int kh_dev_kec256_batch(kh_ctx* c, const uint8_t* d_data, const uint64_t* d_off, uint64_t n, uint8_t* d_out32) {
  if (!c) return set_err(KH_EINVAL, "null context");
  API_TRY({
    HIPCHK(hipSetDevice(c->dev));
    if (n) {
      hipLaunchKernelGGL(k_kec_batch, GRID(n, BS), dim3(BS), 0, c->st, d_data, d_off, n, (uint64_t*)d_out32);
      LAUNCH_CHECK();
    }
  })
}

int kh_kec256_batch(const uint8_t* data, const uint64_t* off, uint64_t n, uint8_t* out32) {
  API_TRY({
    kh_ctx* c = shared_ctx(current_device());
    std::lock_guard<std::recursive_mutex> g(c->mu);
    HIPCHK(hipSetDevice(c->dev));
    if (n == 0) return KH_OK;
    uint64_t o0 = off[0], bytes = off[n] - o0;
    c->in_vals.ensure(bytes + 64);
    c->in_voff.ensure((n + 1) * 8 + 64);
    c->in_keys.ensure(n * 32 + 64);
    std::vector<uint64_t> rel(off, off + n + 1);
    for (auto& x : rel) x -= o0;
    if (bytes) HIPCHK(hipMemcpyAsync(c->in_vals.p, data + o0, bytes, hipMemcpyHostToDevice, c->st));
    HIPCHK(hipMemcpyAsync(c->in_voff.p, rel.data(), (n + 1) * 8, hipMemcpyHostToDevice, c->st));
    hipLaunchKernelGGL(k_kec_batch, GRID(n, BS), dim3(BS), 0, c->st, (const uint8_t*)c->in_vals.p,
                       (const uint64_t*)c->in_voff.p, n, (uint64_t*)c->in_keys.p);
    LAUNCH_CHECK();
    HIPCHK(hipMemcpyAsync(out32, c->in_keys.p, n * 32, hipMemcpyDeviceToHost, c->st));
    HIPCHK(hipStreamSynchronize(c->st));
  })
}

int kh_trie_root(const uint8_t* keys, uint32_t klen, const uint8_t* vals, const uint64_t* voff, uint64_t n,
                 uint32_t flags, uint8_t root32[32], kh_stats* stats) {
  API_TRY({
    if (n && (!keys || !voff)) throw KhError{KH_EINVAL, "null input"};
    if (n == 0) {
      if (stats) memset(stats, 0, sizeof(*stats));
      memcpy(root32, EMPTY_TRIE_HASH, 32);
      return KH_OK;
    }
    kh_ctx* c = shared_ctx(current_device());
    std::lock_guard<std::recursive_mutex> g(c->mu);
    HIPCHK(hipSetDevice(c->dev));
    HostStage H(c);  // the inputs stream in behind the build (keys first)
    Staged S = stage_host_async(c, H, keys, klen, vals, voff, n);
    BuildArgs A{S.keys, klen, S.vals, S.voff, n, nullptr, 1, 0, flags, false};
    A.hs = &H;
    BuildOut O;
    run_build(c, A, O, stats);
    copy_root(O, 0, root32);
  })
}

int kh_trie_roots_segmented(const uint8_t* keys, uint32_t klen, const uint8_t* vals, const uint64_t* voff,
                            const uint64_t* seg_off, uint64_t nseg, uint32_t flags, uint8_t* roots32,
                            kh_stats* stats) {
  API_TRY({
    if (nseg == 0) return KH_OK;
    uint64_t n = seg_off[nseg] - seg_off[0];
    std::vector<uint32_t> seg(n);
    for (uint64_t s = 0; s < nseg; ++s) {
      if (seg_off[s + 1] < seg_off[s]) throw KhError{KH_EINVAL, "seg_off not monotone"};
      for (uint64_t i = seg_off[s]; i < seg_off[s + 1]; ++i) seg[i - seg_off[0]] = (uint32_t)s;
    }
    if (n == 0) {
      for (uint64_t s = 0; s < nseg; ++s) memcpy(roots32 + 32 * s, EMPTY_TRIE_HASH, 32);
      if (stats) memset(stats, 0, sizeof(*stats));
      return KH_OK;
    }
    kh_ctx* c = shared_ctx(current_device());
    std::lock_guard<std::recursive_mutex> g(c->mu);
    HIPCHK(hipSetDevice(c->dev));
    const uint64_t* vo = voff + seg_off[0];
    Staged S = stage_inputs(c, keys + seg_off[0] * klen, klen, vals, vo, n, &seg);
    BuildArgs A{S.keys, klen, S.vals, S.voff, n, S.seg, nseg, 0, flags, false};
    BuildOut O;
    run_build(c, A, O, stats);
    for (uint64_t s = 0; s < nseg; ++s) copy_root(O, s, roots32 + 32 * s);
  })
}

// Variable-length keys (list tries and any unhashed keys of <= 32 bytes): the keys are
// zero-padded on the host to 32 bytes and carry their nibble counts; a key that is a
// prefix of others is the value of the branch at its end (the 17th slot)
int kh_trie_roots_varkeys(const uint8_t* keys, const uint64_t* koff, const uint8_t* vals, const uint64_t* voff,
                          const uint64_t* seg_off, uint64_t nseg, uint8_t* roots32, kh_stats* stats) {
  API_TRY({
    if (nseg == 0) return KH_OK;
    std::vector<uint32_t> seg = seg_ids(seg_off, nseg);
    const uint64_t n = seg.size(), i0 = seg_off[0];
    if (stats) memset(stats, 0, sizeof(*stats));
    if (n == 0) {
      for (uint64_t s = 0; s < nseg; ++s) memcpy(roots32 + 32 * s, EMPTY_TRIE_HASH, 32);
      return KH_OK;
    }
    std::vector<uint8_t> pk(n * 32, 0), kn(n);
    for (uint64_t i = 0; i < n; ++i) {
      const uint64_t a = koff[i0 + i], b = koff[i0 + i + 1];
      if (b < a || b - a > 32) throw KhError{KH_EINVAL, "variable-length keys must be 0..32 bytes"};
      memcpy(&pk[32 * i], keys + a, b - a);
      kn[i] = (uint8_t)(2 * (b - a));
    }
    kh_ctx* c = shared_ctx(current_device());
    std::lock_guard<std::recursive_mutex> g(c->mu);
    HIPCHK(hipSetDevice(c->dev));
    c->in_kn.ensure(n + 64);
    HIPCHK(hipMemcpyAsync(c->in_kn.p, kn.data(), n, hipMemcpyHostToDevice, c->st));
    Staged S = stage_inputs(c, pk.data(), 32, vals, voff + i0, n, nseg > 1 ? &seg : nullptr);
    BuildArgs A{S.keys, 32, S.vals, S.voff, n, S.seg, nseg, 0, 0, false};
    A.kn = (const uint8_t*)c->in_kn.p;
    BuildOut O;
    run_build(c, A, O, stats);
    for (uint64_t s = 0; s < nseg; ++s) copy_root(O, s, roots32 + 32 * s);
  })
}

// List tries (transactions / receipts roots): item i of trie s is keyed by rlp(i), the
// keys generated on the device
int kh_list_roots(const uint8_t* items, const uint64_t* off, const uint64_t* seg_off, uint64_t nseg, uint8_t* roots32,
                  kh_stats* stats) {
  API_TRY({
    if (nseg == 0) return KH_OK;
    std::vector<uint32_t> seg = seg_ids(seg_off, nseg);
    const uint64_t n = seg.size(), i0 = seg_off[0];
    if (stats) memset(stats, 0, sizeof(*stats));
    if (n == 0) {
      for (uint64_t s = 0; s < nseg; ++s) memcpy(roots32 + 32 * s, EMPTY_TRIE_HASH, 32);
      return KH_OK;
    }
    kh_ctx* c = shared_ctx(current_device());
    std::lock_guard<std::recursive_mutex> g(c->mu);
    HIPCHK(hipSetDevice(c->dev));
    c->in_aux.ensure((nseg + 1) * 8 + 64);
    HIPCHK(hipMemcpyAsync(c->in_aux.p, seg_off, (nseg + 1) * 8, hipMemcpyHostToDevice, c->st));
    c->in_kn.ensure(n + 64);
    Staged S = stage_inputs(c, nullptr, 0, items, off + i0, n, &seg);  // keys made below
    c->in_keys.ensure(n * 32 + 64);
    hipLaunchKernelGGL(k_list_keys, GRID(n, BS), dim3(BS), 0, c->st, S.seg, (const uint64_t*)c->in_aux.p, n,
                       (uint64_t*)c->in_keys.p, (uint8_t*)c->in_kn.p);
    LAUNCH_CHECK();
    BuildArgs A{(const uint8_t*)c->in_keys.p, 32, S.vals, S.voff, n, nseg > 1 ? S.seg : nullptr, nseg, 0, 0, false};
    A.kn = (const uint8_t*)c->in_kn.p;
    BuildOut O;
    run_build(c, A, O, stats);
    for (uint64_t s = 0; s < nseg; ++s) copy_root(O, s, roots32 + 32 * s);
  })
}

// kh_list_roots with the items already in HBM (d_off: n + 1 offsets into d_items of the
// n = h_seg_off[nseg] - h_seg_off[0] items; the segment offsets on the host)
int kh_dev_list_roots(kh_ctx* c, const uint8_t* d_items, const uint64_t* d_off, const uint64_t* h_seg_off,
                      uint64_t nseg, uint8_t* roots32, kh_stats* stats) {
  if (!c) return set_err(KH_EINVAL, "null context");
  API_TRY({
    if (nseg == 0) return KH_OK;
    HIPCHK(hipSetDevice(c->dev));
    const uint64_t n = h_seg_off[nseg] - h_seg_off[0];
    if (stats) memset(stats, 0, sizeof(*stats));
    if (n == 0) {
      for (uint64_t s = 0; s < nseg; ++s) memcpy(roots32 + 32 * s, EMPTY_TRIE_HASH, 32);
      return KH_OK;
    }
    hipStream_t st = c->st;
    c->in_aux.ensure((nseg + 1) * 8 + 64);
    c->in_seg.ensure(n * 4 + 64);
    c->in_kn.ensure(n + 64);
    c->in_keys.ensure(n * 32 + 64);
    HIPCHK(hipMemcpyAsync(c->in_aux.p, h_seg_off, (nseg + 1) * 8, hipMemcpyHostToDevice, st));
    hipLaunchKernelGGL(k_seg_ids, GRID(n, BS), dim3(BS), 0, st, (const uint64_t*)c->in_aux.p, nseg, n,
                       (uint32_t*)c->in_seg.p);
    hipLaunchKernelGGL(k_list_keys, GRID(n, BS), dim3(BS), 0, st, (const uint32_t*)c->in_seg.p,
                       (const uint64_t*)c->in_aux.p, n, (uint64_t*)c->in_keys.p, (uint8_t*)c->in_kn.p);
    LAUNCH_CHECK();
    BuildArgs A{(const uint8_t*)c->in_keys.p, 32, d_items, d_off + h_seg_off[0], n,
                nseg > 1 ? (const uint32_t*)c->in_seg.p : nullptr, nseg, 0, 0, false};
    A.kn = (const uint8_t*)c->in_kn.p;
    BuildOut O;
    run_build(c, A, O, stats);
    for (uint64_t s = 0; s < nseg; ++s) copy_root(O, s, roots32 + 32 * s);
  })
}

// Emission of the node set of the build just run on c (c->T): every node reachable from
// the root whose encoding is >= 32 B, plus the root node (MerklePatriciaTrie.scala:505-511),
// restricted to T.emit_sel when set.  Device output in `out`: hashes | rlp | off.
struct EmitLayout {
  uint8_t* hashes;
  uint8_t* rlp;
  uint64_t* off;
};
static EmitLayout emit_layout(DevBuf& out, uint64_t tn, uint64_t tb) {
  uint8_t* oh = (uint8_t*)out.p;
  uint8_t* orlp = oh + ((tn * 32 + 255) & ~255ULL);
  uint64_t* ooff = (uint64_t*)(orlp + ((tb + 255) & ~255ULL));
  return EmitLayout{oh, orlp, ooff};
}
// nodes that are not nodes of the element build appended to a write-back set (the value-only
// branches a commit made): hashes (device, 4 words each), encodings in src at the (offset,
// length) pairs of list (host)
static void em_append(kh_ctx* c, DevBuf& em, uint64_t& tn, uint64_t& tb, const uint64_t* d_hashes, const uint8_t* src,
                      const std::vector<uint64_t>& list) {
  const uint64_t n = list.size() / 2;
  if (!n) return;
  hipStream_t st = c->st;
  uint64_t add = 0;
  for (uint64_t j = 0; j < n; ++j) add += list[2 * j + 1];
  const uint64_t tn2 = tn + n, tb2 = tb + add;
  DevBuf e2;
  e2.ensure(tn2 * 32 + tb2 + (tn2 + 1) * 8 + 1024);
  const EmitLayout A = emit_layout(em, tn, tb), N = emit_layout(e2, tn2, tb2);
  if (tn) HIPCHK(hipMemcpyAsync(N.hashes, A.hashes, tn * 32, hipMemcpyDeviceToDevice, st));
  if (tn) HIPCHK(hipMemcpyAsync(N.off, A.off, tn * 8, hipMemcpyDeviceToDevice, st));
  if (tb) HIPCHK(hipMemcpyAsync(N.rlp, A.rlp, tb, hipMemcpyDeviceToDevice, st));
  HIPCHK(hipMemcpyAsync(N.hashes + tn * 32, d_hashes, n * 32, hipMemcpyDeviceToDevice, st));
  std::vector<uint64_t> offs(n + 1);
  uint64_t at = tb;
  for (uint64_t j = 0; j < n; ++j) {
    HIPCHK(hipMemcpyAsync(N.rlp + at, src + list[2 * j], list[2 * j + 1], hipMemcpyDeviceToDevice, st));
    offs[j] = at;
    at += list[2 * j + 1];
  }
  offs[n] = at;
  HIPCHK(hipMemcpyAsync(N.off + tn, offs.data(), (n + 1) * 8, hipMemcpyHostToDevice, st));
  HIPCHK(hipStreamSynchronize(st));  // (offs is a host temporary)
  swap_buf(em, e2);
  tn = tn2;
  tb = tb2;
}
static int emit_nodes_dev(kh_ctx* c, DevBuf& out, uint64_t* n_nodes, uint64_t* rlp_len) {
  Topo& T = c->T;
  uint64_t B = c->last_B;
  uint64_t Q = T.m + 2 * B;
  // node counts and positions are scanned as uint32
  if (Q >= (1ULL << 32)) throw KhError{KH_EINVAL, "node set too large to emit in one call (>= 2^32 candidates)"};
  c->ws3.ensure(carve_size({Q * 4, Q * 8, Q * 8 + 64}));
  Carver c3{(char*)c->ws3.p, 0, c->ws3.cap};
  uint32_t* flag = c3.take<uint32_t>(Q);
  uint64_t* bytes = c3.take<uint64_t>(Q);
  hipStream_t st = c->st;
  hipLaunchKernelGGL(k_emit_sizes, GRID(Q, BS), dim3(BS), 0, st, T, B, flag, bytes);
  LAUNCH_CHECK();
  uint64_t* totb = (uint64_t*)(T.ctr + CTR_E0);
  uint32_t* totn = (uint32_t*)(T.ctr + CTR_E1);
  HIPCHK(hipMemsetAsync(T.ctr + CTR_E0, 0, 16, st));
  c->out_emit.ensure(scan_scratch_bytes(Q, 8) + 256);
  scan_exclusive<uint64_t>(bytes, bytes, Q, totb, c->out_emit.p, st);
  scan_exclusive<uint32_t>(flag, flag, Q, totn, c->out_emit.p, st);
  HIPCHK(hipMemcpyAsync(c->h_pinned, T.ctr + CTR_E0, 16, hipMemcpyDeviceToHost, st));
  HIPCHK(hipStreamSynchronize(st));
  const uint64_t tb = c->h_pinned[0], tn = (uint32_t)c->h_pinned[1];
  out.ensure(tn * 32 + tb + (tn + 1) * 8 + 1024);
  EmitLayout Lo = emit_layout(out, tn, tb);
  hipLaunchKernelGGL(k_emit_copy, GRID(Q, BS), dim3(BS), 0, st, T, B, (const uint32_t*)flag, (const uint64_t*)bytes,
                     Lo.hashes, Lo.rlp, Lo.off);
  LAUNCH_CHECK();
  c->h_pinned[2] = tb;
  HIPCHK(hipMemcpyAsync(Lo.off + tn, c->h_pinned + 2, 8, hipMemcpyHostToDevice, st));
  HIPCHK(hipStreamSynchronize(st));
  *n_nodes = tn;
  *rlp_len = tb;
  return KH_OK;
}
// host copy of an emitted node set; KH_ENOSPC with the sizes when the caller's buffers are short
static int emit_to_host(kh_ctx* c, DevBuf& src, uint64_t tn, uint64_t tb, uint8_t* hashes32, uint64_t node_cap,
                        uint8_t* rlp, uint64_t rlp_cap, uint64_t* off, uint64_t* n_nodes, uint64_t* rlp_len) {
  *n_nodes = tn;
  *rlp_len = tb;
  if (tn == 0) {  // (no buffer needed: kh_trie_compact may have released it)
    if (off) off[0] = 0;
    return KH_OK;
  }
  if (tn > node_cap || tb > rlp_cap || !hashes32 || !rlp || !off) {
    if (tn == 0 && off) off[0] = 0;
    return (tn == 0) ? KH_OK : set_err(KH_ENOSPC, "output too small");
  }
  EmitLayout Lo = emit_layout(src, tn, tb);
  hipStream_t st = c->st;
  if (tn) HIPCHK(hipMemcpyAsync(hashes32, Lo.hashes, tn * 32, hipMemcpyDeviceToHost, st));
  if (tb) HIPCHK(hipMemcpyAsync(rlp, Lo.rlp, tb, hipMemcpyDeviceToHost, st));
  HIPCHK(hipMemcpyAsync(off, Lo.off, (tn + 1) * 8, hipMemcpyDeviceToHost, st));
  HIPCHK(hipStreamSynchronize(st));
  return KH_OK;
}

int kh_trie_root_nodes(const uint8_t* keys, uint32_t klen, const uint8_t* vals, const uint64_t* voff, uint64_t n,
                       uint32_t flags, uint8_t root32[32], uint8_t* hashes32, uint64_t node_cap, uint8_t* rlp,
                       uint64_t rlp_cap, uint64_t* off, uint64_t* n_nodes, uint64_t* rlp_len, kh_stats* stats) {
  API_TRY({
    *n_nodes = 0;
    *rlp_len = 0;
    if (n == 0) {
      memcpy(root32, EMPTY_TRIE_HASH, 32);
      if (stats) memset(stats, 0, sizeof(*stats));
      if (off && node_cap + 1 > 0) off[0] = 0;
      return KH_OK;
    }
    kh_ctx* c = shared_ctx(current_device());
    std::lock_guard<std::recursive_mutex> g(c->mu);
    HIPCHK(hipSetDevice(c->dev));
    HostStage H(c);  // the inputs stream in behind the build (keys first)
    Staged S = stage_host_async(c, H, keys, klen, vals, voff, n);
    BuildArgs A{S.keys, klen, S.vals, S.voff, n, nullptr, 1, 0, flags, true};
    A.hs = &H;
    BuildOut O;
    run_build(c, A, O, stats);
    copy_root(O, 0, root32);
    uint64_t tn = 0, tb = 0;
    emit_nodes_dev(c, c->emit_dev, &tn, &tb);
    return emit_to_host(c, c->emit_dev, tn, tb, hashes32, node_cap, rlp, rlp_cap, off, n_nodes, rlp_len);
  })
}

int kh_dev_trie_build(kh_ctx* c, const uint8_t* d_keys, uint32_t klen, const uint8_t* d_vals, const uint64_t* d_voff,
                      uint64_t n, const uint32_t* d_seg, uint64_t nseg, uint32_t depth0, uint32_t flags,
                      uint8_t* h_hash32, uint32_t* h_enc_len, uint8_t* h_inline32, kh_stats* stats) {
  return kh_dev_trie_build_ev(c, nullptr, d_keys, klen, d_vals, d_voff, n, d_seg, nseg, depth0, flags, h_hash32,
                              h_enc_len, h_inline32, stats);
}

int kh_dev_trie_build_ev(kh_ctx* c, void* vals_ready, const uint8_t* d_keys, uint32_t klen, const uint8_t* d_vals,
                         const uint64_t* d_voff, uint64_t n, const uint32_t* d_seg, uint64_t nseg, uint32_t depth0,
                         uint32_t flags, uint8_t* h_hash32, uint32_t* h_enc_len, uint8_t* h_inline32,
                         kh_stats* stats) {
  if (!c) return set_err(KH_EINVAL, "null context");
  API_TRY({
    HIPCHK(hipSetDevice(c->dev));
    BuildArgs A{d_keys, klen, d_vals, d_voff, n, d_seg, d_seg ? nseg : 1, depth0, flags, false};
    A.vals_ready = (hipEvent_t)vals_ready;
    static thread_local BuildOut O;  // capacity kept between calls (100k-result builds: no fresh pages)
    run_build(c, A, O, stats);
    uint64_t nres = O.res_len.size();
    if (h_hash32) memcpy(h_hash32, O.res_hash.data(), nres * 32);
    if (h_enc_len) memcpy(h_enc_len, O.res_len.data(), nres * 4);
    if (h_inline32) memcpy(h_inline32, O.res_inl.data(), nres * 32);
  })
}

int kh_fold_root16(const uint8_t* hash32x16, const uint32_t* enc_len16, const uint8_t* inline32x16,
                   uint8_t root32[32]) {
  API_TRY({
    uint64_t refs[64];
    uint32_t lens[16];
    int nonempty = 0;
    for (int i = 0; i < 16; ++i) {
      uint32_t L = enc_len16[i];
      if (L == 0) {
        lens[i] = 0;
        memset(refs + 4 * i, 0, 32);
        continue;
      }
      ++nonempty;
      if (L >= 32) {
        lens[i] = 32;
        memcpy(refs + 4 * i, hash32x16 + 32 * i, 32);
      } else {
        if (!inline32x16) throw KhError{KH_EINVAL, "inline reference without inline bytes"};
        lens[i] = L;
        memcpy(refs + 4 * i, inline32x16 + 32 * i, 32);
      }
    }
    if (nonempty < 2) throw KhError{KH_EINVAL, "fewer than 2 occupied top nibbles: root is not a branch"};
    uint64_t enc[80];  // uint64_t storage: BW stores and Keccak loads are both 8-byte words
    uint32_t L = encode_branch16(refs, lens, (uint8_t*)enc);
    uint64_t h[4];
    kec256_msg<true>((const uint8_t*)enc, L, h);  // host-side Keccak (same code as the device path)
    memcpy(root32, h, 32);
  })
}

int kh_dev_partition(kh_ctx* c, const uint8_t* d_keys32, const uint8_t* d_vals, const uint64_t* d_voff, uint64_t n,
                     uint32_t nparts, uint8_t* d_out_keys, uint8_t* d_out_vals, uint64_t* d_out_vlen,
                     uint64_t* h_counts, uint64_t* h_bytes) {
  return kh_dev_partition_ev(c, nullptr, d_keys32, d_vals, d_voff, n, nparts, d_out_keys, d_out_vals, d_out_vlen,
                             h_counts, h_bytes);
}

// The owner partition; with d_addr (klen-byte keys) the keys are hashed first, in the same
// pass that counts the owners (kh_dev_hash_partition_ev), otherwise d_keys32 are the keys
static void partition_impl(kh_ctx* c, void* vals_done, const uint8_t* d_addr, uint32_t klen, const uint8_t* d_keys32,
                           const uint8_t* d_vals, const uint64_t* d_voff, uint64_t n, uint32_t nparts,
                           uint8_t* d_out_keys, uint8_t* d_out_vals, uint64_t* d_out_vlen, uint64_t* h_counts,
                           uint64_t* h_bytes) {
  {
    if (nparts < 1 || nparts > 16) throw KhError{KH_EINVAL, "nparts must be in [1, 16]"};
    if (d_addr && (klen == 0 || klen > 4096)) throw KhError{KH_EINVAL, "bad key length"};
    HIPCHK(hipSetDevice(c->dev));
    memset(h_counts, 0, nparts * 8);
    memset(h_bytes, 0, nparts * 8);
    if (n == 0) {  // nothing to copy: vals_done is still recorded, as khst.h promises
      if (vals_done) HIPCHK(hipEventRecord((hipEvent_t)vals_done, c->st));
      return;
    }
    if (n >= (1ULL << 31)) throw KhError{KH_EINVAL, "n must be < 2^31 per device"};
    if ((uintptr_t)d_keys32 & 7 || (uintptr_t)d_out_keys & 7 || (uintptr_t)d_voff & 7 || (uintptr_t)d_out_vlen & 7 ||
        (uintptr_t)d_out_vals & 7)
      throw KhError{KH_EINVAL, "partition: keys, offsets, lengths and the value output must be 8-byte aligned"};
    hipStream_t st = c->st;
    const uint32_t ntile = (uint32_t)((n + PT_TILE - 1) / PT_TILE);
    const uint64_t nh = (uint64_t)nparts * ntile;
    c->ws3.ensure(carve_size({nh * 4, n * 4, n * 8, scan_scratch_bytes(std::max<uint64_t>(n, nh), 8), 40 * 8,
                              d_addr ? n * 32 : 0, nh * 8, d_addr ? n + 16 : 0}));
    Carver cv{(char*)c->ws3.p, 0, c->ws3.cap};
    uint32_t* hist = cv.take<uint32_t>(nh);
    uint32_t* pos = cv.take<uint32_t>(n);
    uint64_t* ooff = cv.take<uint64_t>(n);
    void* sc = cv.take<char>(scan_scratch_bytes(std::max<uint64_t>(n, nh), 8));
    unsigned long long* tot = cv.take<unsigned long long>(40);  // counts | bytes | byte total
    const uint64_t* K = (const uint64_t*)d_keys32;
    // the place pass sums the tiles' value bytes per owner: the counts and bytes go back to the
    // host before the scan of the placed lengths (that scan, and with vals_done the value copy,
    // run after the return)
    unsigned long long* hbytes = cv.take<unsigned long long>(nh);
    if (d_addr) {  // hashed here, each owner written as a byte that the count pass reads
      uint64_t* hk = cv.take<uint64_t>(n * 4);
      uint8_t* ob = cv.take<uint8_t>(n + 16);
      if (klen <= 135)
        hipLaunchKernelGGL(k_hash_keys_owner_s, GRID(n, BS), dim3(BS), 0, st, d_addr, klen, n, hk, nparts, ob);
      else
        hipLaunchKernelGGL(k_hash_keys_owner_l, GRID(n, BS), dim3(BS), 0, st, d_addr, klen, n, hk, nparts, ob);
      LAUNCH_CHECK();
      hipLaunchKernelGGL(k_part_count_o, dim3(ntile), dim3(BS), 0, st, (const uint8_t*)ob, n, nparts, ntile, hist);
      LAUNCH_CHECK();
      K = hk;
    } else {
      hipLaunchKernelGGL(k_part_count, dim3(ntile), dim3(BS), 0, st, K, n, nparts, ntile, hist);
      LAUNCH_CHECK();
    }
    scan_exclusive<uint32_t>(hist, hist, nh, (uint32_t*)nullptr, sc, st);
    if (!(((uintptr_t)K | (uintptr_t)d_out_keys) & 15))
      hipLaunchKernelGGL(k_part_place<true>, dim3(ntile), dim3(BS), 0, st, K, d_voff, n, nparts, ntile,
                         (const uint32_t*)hist, (uint64_t*)d_out_keys, d_out_vlen, pos, hbytes);
    else
      hipLaunchKernelGGL(k_part_place<false>, dim3(ntile), dim3(BS), 0, st, K, d_voff, n, nparts, ntile,
                         (const uint32_t*)hist, (uint64_t*)d_out_keys, d_out_vlen, pos, hbytes);
    LAUNCH_CHECK();
    auto vcopy = [&] {
      scan_exclusive<uint64_t>(d_out_vlen, ooff, n, (uint64_t*)(tot + 32), sc, st);
      hipLaunchKernelGGL(k_part_vcopy, GRID(n * CG, BS), dim3(BS), 0, st, d_vals, d_voff, (const uint32_t*)pos,
                         (const uint64_t*)ooff, n, d_out_vals);
      LAUNCH_CHECK();
    };
    if (!vals_done) vcopy();
    hipLaunchKernelGGL(k_part_bounds_t, dim3(nparts), dim3(BS), 0, st, (const uint32_t*)hist,
                       (const unsigned long long*)hbytes, ntile, n, nparts, tot, tot + 16);
    LAUNCH_CHECK();
    HIPCHK(hipMemcpyAsync(c->h_pinned, tot, 256, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    if (vals_done) {  // the value bytes move after the counts are back: the caller routes the
                      // keys meanwhile and orders the value exchange after vals_done
      vcopy();
      HIPCHK(hipEventRecord((hipEvent_t)vals_done, st));
    }
    for (uint32_t p = 0; p < nparts; ++p) {
      h_counts[p] = c->h_pinned[p];
      h_bytes[p] = c->h_pinned[16 + p];
    }
  }
}
int kh_dev_partition_ev(kh_ctx* c, void* vals_done, const uint8_t* d_keys32, const uint8_t* d_vals,
                        const uint64_t* d_voff, uint64_t n, uint32_t nparts, uint8_t* d_out_keys,
                        uint8_t* d_out_vals, uint64_t* d_out_vlen, uint64_t* h_counts, uint64_t* h_bytes) {
  if (!c) return set_err(KH_EINVAL, "null context");
  API_TRY({
    partition_impl(c, vals_done, nullptr, 0, d_keys32, d_vals, d_voff, n, nparts, d_out_keys, d_out_vals, d_out_vlen,
                   h_counts, h_bytes);
  })
}
int kh_dev_hash_partition_ev(kh_ctx* c, void* vals_done, const uint8_t* d_keys, uint32_t klen, const uint8_t* d_vals,
                             const uint64_t* d_voff, uint64_t n, uint32_t nparts, uint8_t* d_out_keys,
                             uint8_t* d_out_vals, uint64_t* d_out_vlen, uint64_t* h_counts, uint64_t* h_bytes) {
  if (!c) return set_err(KH_EINVAL, "null context");
  API_TRY({
    if (n && !d_keys) throw KhError{KH_EINVAL, "null keys"};
    partition_impl(c, vals_done, d_keys, klen, nullptr, d_vals, d_voff, n, nparts, d_out_keys, d_out_vals,
                   d_out_vlen, h_counts, h_bytes);
  })
}

int kh_dev_hash_keys(kh_ctx* c, const uint8_t* d_keys, uint32_t klen, uint64_t n, uint8_t* d_out32) {
  if (!c) return set_err(KH_EINVAL, "null context");
  API_TRY({
    HIPCHK(hipSetDevice(c->dev));
    if (n) {
      if (klen <= 135)
        hipLaunchKernelGGL(k_hash_keys<true>, GRID(n, BS), dim3(BS), 0, c->st, d_keys, klen, n, (uint64_t*)d_out32);
      else
        hipLaunchKernelGGL(k_hash_keys<false>, GRID(n, BS), dim3(BS), 0, c->st, d_keys, klen, n, (uint64_t*)d_out32);
      LAUNCH_CHECK();
    }
  })
}

// ---- synthetic storage tries (csrc/synth.h): slot counts, slot value lengths, slots
__global__ void __launch_bounds__(BS) k_st_count(uint32_t cfg, uint64_t t0, uint64_t nt, uint64_t* cnt) {
  const uint64_t t = (uint64_t)blockIdx.x * BS + threadIdx.x;
  if (t <= nt) cnt[t] = t < nt ? synth_storage_slots(cfg, t0 + t) : 0;
}
__global__ void __launch_bounds__(BS) k_st_vlen(uint32_t cfg, uint64_t t0, const uint64_t* seg_off, const uint32_t* seg,
                                                uint64_t n, uint64_t* vlen) {
  const uint64_t i = (uint64_t)blockIdx.x * BS + threadIdx.x;
  if (i > n) return;
  if (i == n) {
    vlen[n] = 0;
    return;
  }
  const uint32_t t = seg[i];
  vlen[i] = synth_slot(cfg, t0 + t, (uint32_t)(i - seg_off[t])).enc;
}
__global__ void __launch_bounds__(BS) k_st_write(uint32_t cfg, uint64_t t0, const uint64_t* seg_off, const uint32_t* seg,
                                                 uint64_t n, const uint64_t* voff, uint8_t* keys, uint8_t* vals) {
  const uint64_t i = (uint64_t)blockIdx.x * BS + threadIdx.x;
  if (i >= n) return;
  const uint32_t t = seg[i], slot = (uint32_t)(i - seg_off[t]);
  synth_slot_write(synth_slot(cfg, t0 + t, slot), slot, keys + 32 * i, vals + voff[i]);
}

int kh_dev_synth_storage(kh_ctx* c, uint32_t cfg, uint64_t t0, uint64_t nt, uint64_t* d_seg_off, uint64_t* n_slots,
                         uint64_t* val_bytes, uint8_t* d_keys, uint8_t* d_vals, uint64_t* d_voff, uint32_t* d_seg) {
  if (!c) return set_err(KH_EINVAL, "null context");
  if (!d_seg_off || !n_slots || !val_bytes) return set_err(KH_EINVAL, "null output");
  API_TRY({
    HIPCHK(hipSetDevice(c->dev));
    hipStream_t st = c->st;
    if (nt >= (1ULL << 31)) throw KhError{KH_EINVAL, "too many tries"};
    hipLaunchKernelGGL(k_st_count, GRID(nt + 1, BS), dim3(BS), 0, st, cfg, t0, nt, d_seg_off);
    LAUNCH_CHECK();
    c->out_emit.ensure(scan_scratch_bytes(nt + 1, 8) + 256);
    scan_exclusive<uint64_t>(d_seg_off, d_seg_off, nt + 1, (uint64_t*)nullptr, c->out_emit.p, st);
    HIPCHK(hipMemcpyAsync(c->h_pinned, d_seg_off + nt, 8, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    const uint64_t n = c->h_pinned[0];
    if (n >= (1ULL << 31)) throw KhError{KH_EINVAL, "more than 2^31 slots"};
    *n_slots = n;
    const bool write = d_keys != nullptr;
    if (write && (!d_vals || !d_voff || !d_seg)) throw KhError{KH_EINVAL, "null output"};
    c->ws3.ensure(carve_size({n * 4 + 64, (n + 1) * 8 + 64}));
    Carver cv{(char*)c->ws3.p, 0, c->ws3.cap};
    uint32_t* seg = write ? d_seg : cv.take<uint32_t>(n + 16);
    uint64_t* vo = write ? d_voff : cv.take<uint64_t>(n + 1);
    if (n) {
      hipLaunchKernelGGL(k_seg_ids, GRID(n, BS), dim3(BS), 0, st, (const uint64_t*)d_seg_off, nt, n, seg);
      LAUNCH_CHECK();
    }
    hipLaunchKernelGGL(k_st_vlen, GRID(n + 1, BS), dim3(BS), 0, st, cfg, t0, (const uint64_t*)d_seg_off,
                       (const uint32_t*)seg, n, vo);
    LAUNCH_CHECK();
    c->out_emit.ensure(scan_scratch_bytes(n + 1, 8) + 256);
    scan_exclusive<uint64_t>(vo, vo, n + 1, (uint64_t*)nullptr, c->out_emit.p, st);
    HIPCHK(hipMemcpyAsync(c->h_pinned, vo + n, 8, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    *val_bytes = c->h_pinned[0];
    if (write && n) {
      hipLaunchKernelGGL(k_st_write, GRID(n, BS), dim3(BS), 0, st, cfg, t0, (const uint64_t*)d_seg_off,
                         (const uint32_t*)seg, n, (const uint64_t*)vo, d_keys, d_vals);
      LAUNCH_CHECK();
      HIPCHK(hipStreamSynchronize(st));
    }
  })
}

int kh_dev_synth_accounts(kh_ctx* c, uint32_t cfg, uint64_t first, uint64_t n, uint8_t* d_addr, uint8_t* d_vals,
                          uint64_t* d_voff) {
  if (!c) return set_err(KH_EINVAL, "null context");
  API_TRY({
    HIPCHK(hipSetDevice(c->dev));
    if (n == 0) {
      HIPCHK(hipMemsetAsync(d_voff, 0, 8, c->st));
      return KH_OK;
    }
    hipStream_t st = c->st;
    hipLaunchKernelGGL(k_synth_len, GRID(n + 1, BS), dim3(BS), 0, st, cfg, first, n, d_voff);
    LAUNCH_CHECK();
    c->out_emit.ensure(scan_scratch_bytes(n + 1, 8) + 256);
    scan_exclusive<uint64_t>(d_voff, d_voff, n + 1, (uint64_t*)nullptr, c->out_emit.p, st);
    hipLaunchKernelGGL(k_synth_write, GRID(n, BS), dim3(BS), 0, st, cfg, first, n, (const uint64_t*)d_voff, d_addr,
                       d_vals);
    LAUNCH_CHECK();
    HIPCHK(hipStreamSynchronize(st));
  })
}

// NodeDatasRequest.processResponse over one batch: the values and requests staged,
// the requests sorted and deduplicated on the device (the last of equal hashes wins), every value
// hashed, matched and decoded by k_verify_nodes, the children packed; one host sync.  Outputs
// through the context's pinned staging.  packed: child_off[n+1] + packed children; else the
// 16-slot rows of kh_verify_nodes.
static int verify_nodes_impl(const uint8_t* data, const uint64_t* off, uint64_t n, const uint8_t* req32,
                             const uint8_t* req_kind, uint64_t nreq, uint8_t* hash32, int64_t* match, uint8_t* status,
                             uint8_t* nchild_rows, uint8_t* child_rows, uint8_t* kind_rows, uint64_t* child_off,
                             uint8_t* child32, uint8_t* child_kind, uint64_t child_cap, uint64_t* n_children) {
  if (n_children) *n_children = 0;
  if (n == 0) {
    if (child_off) child_off[0] = 0;
    return KH_OK;
  }
  if (!data || !off || (nreq && (!req32 || !req_kind))) throw KhError{KH_EINVAL, "null buffer"};
  if (n >= (1ULL << 31) || nreq >= (1ULL << 31)) throw KhError{KH_EINVAL, "batch too large"};
  kh_ctx* c = shared_ctx(current_device());
  std::lock_guard<std::recursive_mutex> g(c->mu);
  HIPCHK(hipSetDevice(c->dev));
  hipStream_t st = c->st;
  const uint64_t v0 = off[0], vbytes = off[n] - v0;
  std::vector<uint64_t> rel(off, off + n + 1);
  for (auto& x : rel) x -= v0;
  c->in_vals.ensure(vbytes + 64);
  c->in_voff.ensure((n + 1) * 8 + 64);
  const uint64_t nr = nreq ? nreq : 1;
  c->in_keys.ensure(carve_size({32 * nr + 32, nr + 1}));
  Carver ci{(char*)c->in_keys.p, 0, c->in_keys.cap};
  uint64_t* dreq = ci.take<uint64_t>(4 * nr + 4);
  uint8_t* dkind = ci.take<uint8_t>(nr + 1);
  if (vbytes) HIPCHK(hipMemcpyAsync(c->in_vals.p, data + v0, vbytes, hipMemcpyHostToDevice, st));
  HIPCHK(hipMemcpyAsync(c->in_voff.p, rel.data(), (n + 1) * 8, hipMemcpyHostToDevice, st));
  if (nreq) {
    HIPCHK(hipMemcpyAsync(dreq, req32, 32 * nreq, hipMemcpyHostToDevice, st));
    HIPCHK(hipMemcpyAsync(dkind, req_kind, nreq, hipMemcpyHostToDevice, st));
  }
  // the requests in key order, one per distinct hash (sort_dedup: the last duplicate kept)
  c->ws1.ensure(carve_size({nr * 8, nr * 8, nr * 4, nr * 4, nr * 32, radix_scratch_bytes(nr),
                            scan_scratch_bytes(nr, 8), CTR_N * 8}));
  Carver cs{(char*)c->ws1.p, 0, c->ws1.cap};
  SortIO S{(const uint64_t*)dreq, nullptr, 0, nreq, cs.take<uint64_t>(nr), cs.take<uint64_t>(nr),
           cs.take<uint32_t>(nr), cs.take<uint32_t>(nr), cs.take<uint64_t>(nr * 4), nullptr,
           cs.take<char>(radix_scratch_bytes(nr)), cs.take<char>(scan_scratch_bytes(nr, 8)),
           cs.take<unsigned long long>(CTR_N), nullptr, false};
  uint64_t m = 0;
  const uint64_t* skey = dreq;
  const uint32_t* sidx = nullptr;
  if (nreq) {
    HIPCHK(hipMemsetAsync(S.ctr, 0, CTR_N * 8, st));
    if (nreq == 1) {  // (nothing to sort)
      HIPCHK(hipMemsetAsync(S.idx0, 0, 4, st));
      m = 1;
      sidx = S.idx0;
    } else {
      sort_dedup(c, S);
      m = S.m;
      skey = S.skey;
      sidx = S.sidx;
    }
  }
  // per value: hash, match, decode (16-slot rows), then the children packed
  c->out_emit.ensure(carve_size({32 * n, 8 * n, n, 4 * n, 512 * n, 16 * n, 8 * (n + 1), scan_scratch_bytes(n + 1, 8),
                                 32 * 16 * n, 16 * n, 64}));
  Carver co{(char*)c->out_emit.p, 0, c->out_emit.cap};
  uint64_t* dh = co.take<uint64_t>(4 * n);
  int64_t* dm = co.take<int64_t>(n);
  uint8_t* ds = co.take<uint8_t>(n);
  uint32_t* dn = co.take<uint32_t>(n);
  uint8_t* dc = co.take<uint8_t>(512 * n);
  uint8_t* dk = co.take<uint8_t>(16 * n);
  uint64_t* coff = co.take<uint64_t>(n + 1);
  void* sscr = co.take<char>(scan_scratch_bytes(n + 1, 8));
  uint8_t* pc = co.take<uint8_t>(32 * 16 * n);
  uint8_t* pk = co.take<uint8_t>(16 * n);
  uint64_t* tot = co.take<uint64_t>(8);
  hipLaunchKernelGGL(k_verify_nodes, GRID(n, BS), dim3(BS), 0, st, (const uint8_t*)c->in_vals.p,
                     (const uint64_t*)c->in_voff.p, n, skey, (const uint8_t*)dkind, sidx, m, dh, dm, ds, dn, dc, dk);
  LAUNCH_CHECK();
  // (counts widened: scan_exclusive sums 64-bit offsets from 32-bit counts through a copy)
  hipLaunchKernelGGL(k_u32_to_u64, GRID(n, BS), dim3(BS), 0, st, (const uint32_t*)dn, n, coff);
  LAUNCH_CHECK();
  scan_exclusive<uint64_t>(coff, coff, n, tot, sscr, st);
  hipLaunchKernelGGL(k_set_last, dim3(1), dim3(1), 0, st, coff + n, (const uint64_t*)tot);
  hipLaunchKernelGGL(k_pack_children, GRID(16 * n, BS), dim3(BS), 0, st, (const uint32_t*)dn, (const uint64_t*)coff, n,
                     (const uint8_t*)dc, (const uint8_t*)dk, pc, pk);
  LAUNCH_CHECK();
  HIPCHK(hipMemcpyAsync(c->h_pinned, tot, 8, hipMemcpyDeviceToHost, st));
  HIPCHK(hipStreamSynchronize(st));
  const uint64_t total = c->h_pinned[0];
  if (n_children) *n_children = total;
  // outputs through pinned staging: hashes, matches, statuses, counts / offsets, children
  const uint64_t bytes = 32 * n + 8 * n + n + 8 * (n + 1) + 4 * n + 33 * total + 64;
  uint8_t* hs = pinned_stage(c, bytes);
  uint8_t* hp = hs;
  auto back = [&](void* dst, const void* src, uint64_t b) {
    if (!dst || !b) return;
    HIPCHK(hipMemcpyAsync(hp, src, b, hipMemcpyDeviceToHost, st));
    hp += b;
  };
  uint8_t *h_hash = hp;
  back(hash32, dh, 32 * n);
  uint8_t* h_match = hp;
  back(match, dm, 8 * n);
  uint8_t* h_status = hp;
  back(status, ds, n);
  uint8_t* h_coff = hp;
  back((void*)1, coff, 8 * (n + 1));
  uint8_t* h_pc = hp;
  back((void*)1, pc, 32 * total);
  uint8_t* h_pk = hp;
  back((void*)1, pk, total);
  HIPCHK(hipStreamSynchronize(st));
  if (hash32) memcpy(hash32, h_hash, 32 * n);
  if (match) memcpy(match, h_match, 8 * n);
  if (status) memcpy(status, h_status, n);
  const uint64_t* hco = (const uint64_t*)h_coff;
  if (child_off) {  // packed
    memcpy(child_off, hco, 8 * (n + 1));
    if (total > child_cap || (total && (!child32 || !child_kind)))
      return set_err(KH_ENOSPC, "children output too small");
    memcpy(child32, h_pc, 32 * total);
    memcpy(child_kind, h_pk, total);
  } else {  // the 16-slot rows of kh_verify_nodes
    for (uint64_t i = 0; i < n; ++i) {
      const uint64_t a = hco[i], k = hco[i + 1] - a;
      if (nchild_rows) nchild_rows[i] = (uint8_t)k;
      if (k && child_rows) memcpy(child_rows + 512 * i, h_pc + 32 * a, 32 * k);
      if (k && kind_rows) memcpy(kind_rows + 16 * i, h_pk + a, k);
    }
  }
  return KH_OK;
}

int kh_verify_nodes(const uint8_t* data, const uint64_t* off, uint64_t n, const uint8_t* req32, const uint8_t* req_kind,
                    uint64_t nreq, uint8_t* hash32, int64_t* match, uint8_t* status, uint8_t* nchild, uint8_t* child32,
                    uint8_t* child_kind) {
  API_TRY({
    return verify_nodes_impl(data, off, n, req32, req_kind, nreq, hash32, match, status, nchild, child32, child_kind,
                             nullptr, nullptr, nullptr, 0, nullptr);
  })
}
int kh_verify_nodes_packed(const uint8_t* data, const uint64_t* off, uint64_t n, const uint8_t* req32,
                           const uint8_t* req_kind, uint64_t nreq, uint8_t* hash32, int64_t* match, uint8_t* status,
                           uint64_t* child_off, uint8_t* child32, uint8_t* child_kind, uint64_t child_cap,
                           uint64_t* n_children) {
  if (!child_off) return set_err(KH_EINVAL, "null child offsets");
  API_TRY({
    return verify_nodes_impl(data, off, n, req32, req_kind, nreq, hash32, match, status, nullptr, nullptr, nullptr,
                             child_off, child32, child_kind, child_cap, n_children);
  })
}

static OItems oitems_carve(DevBuf& b, uint64_t cap) {
  b.ensure(carve_size({cap * 32, cap, cap, cap * 32, cap, cap * 32, cap, 64}));
  Carver cv{(char*)b.p, 0, b.cap};
  OItems I{};
  I.pre = cv.take<uint64_t>(cap * 4);
  I.a = cv.take<uint8_t>(cap);
  I.d = cv.take<uint8_t>(cap);
  I.ref = cv.take<uint64_t>(cap * 4);
  I.rl = cv.take<uint8_t>(cap);
  I.pref = cv.take<uint64_t>(cap * 4);
  I.prl = cv.take<uint8_t>(cap);
  I.n = cv.take<unsigned long long>(8);
  I.cap = cap;
  return I;
}

// open an (empty) trie from root32 and n stored node encodings (device buffers)
static void trie_open_nodes(kh_trie* h, const uint8_t* root32, const uint8_t* d_enc, const uint64_t* d_off,
                            uint64_t n, uint8_t* missing32) {
  kh_ctx* c = h->c;
  hipStream_t st = c->st;
  memcpy(h->root, root32, 32);
  if (memcmp(root32, EMPTY_TRIE_HASH, 32) == 0) return;  // MerklePatriciaTrie.scala:60-66
  if (n >= (1ULL << 31)) throw KhError{KH_EINVAL, "node store too large"};
  // the store, keyed by kec256 of each encoding (content addressed)
  std::vector<size_t> sz = {n * 32 + 32, n * 8, n * 8, n * 4, n * 4, n * 32 + 32, radix_scratch_bytes(n + 1),
                            scan_scratch_bytes(n + 1, 8), CTR_N * 8, 64, 64};
  h->ws.ensure(carve_size(sz));
  Carver cv{(char*)h->ws.p, 0, h->ws.cap};
  uint64_t* hs = cv.take<uint64_t>(n * 4 + 4);
  SortIO S{};
  S.K32 = hs;
  S.n = n;
  S.ck0 = cv.take<uint64_t>(n);
  S.ck1 = cv.take<uint64_t>(n);
  S.idx0 = cv.take<uint32_t>(n);
  S.idx1 = cv.take<uint32_t>(n);
  S.skey = cv.take<uint64_t>(n * 4 + 4);
  S.rs_scratch = cv.take<char>(radix_scratch_bytes(n + 1));
  S.scan_scratch = cv.take<char>(scan_scratch_bytes(n + 1, 8));
  S.ctr = cv.take<unsigned long long>(CTR_N);
  unsigned long long* oc = cv.take<unsigned long long>(8);  // records, heap bytes, leaves, error
  uint8_t* dmiss = cv.take<uint8_t>(64);
  HIPCHK(hipMemsetAsync(S.ctr, 0, CTR_N * 8, st));
  HIPCHK(hipMemsetAsync(oc, 0, 64, st));
  uint64_t total = 0;
  NStore NS{nullptr, nullptr, 0, d_enc, d_off};
  if (n) {
    hipLaunchKernelGGL(k_kec_batch, GRID(n, BS), dim3(BS), 0, st, d_enc, d_off, n, hs);
    LAUNCH_CHECK();
    sort_dedup(c, S);
    NS.hash = S.skey;
    NS.idx = S.sidx;
    NS.m = S.m;
    HIPCHK(hipMemcpyAsync(c->h_pinned, d_off, 8, hipMemcpyDeviceToHost, st));
    HIPCHK(hipMemcpyAsync(c->h_pinned + 1, d_off + n, 8, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    total = c->h_pinned[1] - c->h_pinned[0];
  }
  // leaf values land in the heap: at most the store's bytes
  regrow(h->heap, h->heap_n, h->heap_n + total + 64, st);
  c->h_pinned[0] = h->heap_n;
  HIPCHK(hipMemcpyAsync(oc + 1, c->h_pinned, 8, hipMemcpyHostToDevice, st));
  DevBuf fa, fb;
  OItems cur = oitems_carve(fa, 1);
  {  // the root: referenced by its hash, at anchor 0
    uint64_t w[4];
    memcpy(w, root32, 32);
    c->h_pinned[1] = 1;
    HIPCHK(hipMemsetAsync(cur.pre, 0, 32, st));
    HIPCHK(hipMemsetAsync(cur.a, 0, 1, st));
    HIPCHK(hipMemsetAsync(cur.d, 0, 1, st));
    HIPCHK(hipMemcpyAsync(cur.ref, w, 32, hipMemcpyHostToDevice, st));
    HIPCHK(hipMemcpyAsync(cur.pref, w, 32, hipMemcpyHostToDevice, st));
    HIPCHK(hipMemsetAsync(cur.rl, 32, 1, st));
    HIPCHK(hipMemsetAsync(cur.prl, 32, 1, st));
    HIPCHK(hipStreamSynchronize(st));  // w is a host temporary
  }
  uint64_t ni = 1, nrec = 0;
  const uint64_t rn0 = h->rn;
  for (int level = 0; ni && level < 80; ++level) {
    h->rn = rn0 + nrec;  // a regrow keeps the records of the earlier levels
    recs_reserve(h, h->rn + ni + 16);
    OItems nxt = oitems_carve(level & 1 ? fa : fb, 16 * ni);
    HIPCHK(hipMemsetAsync(nxt.n, 0, 8, st));
    hipLaunchKernelGGL(k_open_level, GRID(ni, BS), dim3(BS), 0, st, cur, ni, nxt, NS, recs_of(h), oc, rn0,
                       0u, (uint8_t*)h->heap.p, oc + 1, oc + 2, oc + 3, dmiss);
    LAUNCH_CHECK();
    HIPCHK(hipMemcpyAsync(c->h_pinned, nxt.n, 8, hipMemcpyDeviceToHost, st));
    HIPCHK(hipMemcpyAsync(c->h_pinned + 1, oc, 32, hipMemcpyDeviceToHost, st));
    HIPCHK(hipMemcpyAsync(c->h_pinned + 8, dmiss, 32, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    const uint64_t code = c->h_pinned[4];
    if (code == OPEN_MISSING) {
      if (missing32) memcpy(missing32, c->h_pinned + 8, 32);
      throw KhError{KH_ENODE, "node missing from the store (MPTNodeMissingException)"};
    }
    if (code == OPEN_VALUE) throw KhError{KH_EINVAL, "a branch with a value: not a secure trie"};
    if (code) throw KhError{KH_EINVAL, "the store holds a node that is not a canonical secure-trie node"};
    nrec = c->h_pinned[1];
    ni = c->h_pinned[0];
    cur = nxt;
  }
  if (ni) throw KhError{KH_EINVAL, "node store deeper than a 32-byte key allows"};
  h->rn = rn0 + nrec;
  h->heap_n = c->h_pinned[2];
  h->nleaves += c->h_pinned[3];
  map_rebuild(h, 1024);
}

static kh_trie* trie_new(kh_ctx* c, uint32_t flags, bool forest) {
  kh_trie* h = new kh_trie();
  h->c = c;
  h->home = c;
  h->lk = &c->mu;
  h->flags = flags;
  h->forest = forest;
  memcpy(h->root, EMPTY_TRIE_HASH, 32);
  return h;
}
// a handle of the shared context moves to a private one (kh_trie::priv) once its open has
// completed on the shared context (its in-flight tail drained first: the private streams are
// not ordered after the shared one)
static void make_private(kh_trie* h) {
  if (h->priv) return;
  trie_settle(h);
  HIPCHK(hipStreamSynchronize(h->c->st));
  HIPCHK(hipStreamSynchronize(h->c->st2));
  h->priv = ctx_new(h->home->dev);
  h->c = h->priv;
  h->lk = &h->own_mu;
}
static void check_flags(const kh_trie* h, uint32_t flags) {
  if ((flags & KH_HASH_KEYS) != (h->flags & KH_HASH_KEYS))
    throw KhError{KH_EINVAL, "KH_HASH_KEYS differs from the flag the trie was opened with"};
}

int kh_trie_open(kh_ctx* c, const uint8_t* d_keys, uint32_t klen, const uint8_t* d_vals, const uint64_t* d_voff,
                 uint64_t n, uint32_t flags, uint8_t root32[32], kh_trie** out) {
  if (!c || !out) return set_err(KH_EINVAL, "null context or handle");
  std::lock_guard<std::recursive_mutex> g(c->mu);
  kh_trie* h = nullptr;
  API_TRY({
    HIPCHK(hipSetDevice(c->dev));
    h = trie_new(c, flags, false);
    try {
      FCommit F;
      F.up_keys = d_keys;
      F.up_vals = d_vals;
      F.up_voff = d_voff;
      F.nup = n;
      F.klen = klen;
      forest_commit(h, F, nullptr);
    } catch (...) {
      delete h;
      h = nullptr;
      throw;
    }
    if (root32) memcpy(root32, h->root, 32);
    *out = h;
  })
}

int kh_trie_open_nodes(kh_ctx* c, const uint8_t root32[32], const uint8_t* d_enc, const uint64_t* d_off, uint64_t n,
                       uint32_t flags, uint8_t missing32[32], kh_trie** out) {
  if (!c || !out || !root32) return set_err(KH_EINVAL, "null context, root or handle");
  std::lock_guard<std::recursive_mutex> g(c->mu);
  kh_trie* h = nullptr;
  API_TRY({
    HIPCHK(hipSetDevice(c->dev));
    h = trie_new(c, flags, false);
    try {
      trie_open_nodes(h, root32, d_enc, d_off, n, missing32);
    } catch (...) {
      delete h;
      h = nullptr;
      throw;
    }
    *out = h;
  })
}

int kh_trie_open_nodes_host(const uint8_t root32[32], const uint8_t* enc, const uint64_t* off, uint64_t n,
                            uint32_t flags, uint8_t missing32[32], kh_trie** out) {
  if (!out || !root32 || (n && (!enc || !off))) return set_err(KH_EINVAL, "null input");
  API_TRY({
    kh_ctx* c = shared_ctx(current_device());
    std::lock_guard<std::recursive_mutex> g(c->mu);
    HIPCHK(hipSetDevice(c->dev));
    const uint64_t o0 = n ? off[0] : 0, bytes = n ? off[n] - o0 : 0;
    c->in_vals.ensure(bytes + 64);
    c->in_voff.ensure((n + 1) * 8 + 64);
    std::vector<uint64_t> rel(n + 1, 0);
    for (uint64_t i = 0; i <= n && n; ++i) rel[i] = off[i] - o0;
    if (bytes) HIPCHK(hipMemcpyAsync(c->in_vals.p, enc + o0, bytes, hipMemcpyHostToDevice, c->st));
    HIPCHK(hipMemcpyAsync(c->in_voff.p, rel.data(), (n + 1) * 8, hipMemcpyHostToDevice, c->st));
    HIPCHK(hipStreamSynchronize(c->st));
    int rc = kh_trie_open_nodes(c, root32, (const uint8_t*)c->in_vals.p, (const uint64_t*)c->in_voff.p, n, flags,
                                missing32, out);
    if (rc != KH_OK) return rc;
    try {
      make_private(*out);
    } catch (...) {
      delete *out;
      *out = nullptr;
      throw;
    }
  })
}

int kh_trie_open_host(const uint8_t* keys, uint32_t klen, const uint8_t* vals, const uint64_t* voff, uint64_t n,
                      uint32_t flags, uint8_t root32[32], kh_trie** out) {
  if (!out || (n && (!keys || !voff))) return set_err(KH_EINVAL, "null input");
  API_TRY({
    kh_ctx* c = shared_ctx(current_device());
    std::lock_guard<std::recursive_mutex> g(c->mu);
    HIPCHK(hipSetDevice(c->dev));
    static const uint64_t zero_off[1] = {0};
    if (n == 0) voff = zero_off;
    // the inputs stream in behind the open's commit: its op pass reads the keys and offsets, the
    // values are waited for where the commit first copies them (FCommit::before_values)
    HostStage H(c);
    Staged S = stage_host_async(c, H, keys, klen, vals, voff, n);
    H.stream_wait(c->st, H.nkp);
    kh_trie* h = trie_new(c, flags, false);
    try {
      FCommit F;
      F.up_keys = S.keys;
      F.up_vals = S.vals;
      F.up_voff = S.voff;
      F.nup = n;
      F.klen = klen;
      F.before_values = [&H] { H.wait(H.nkp + 1); };
      F.vals_ready = H.ev(H.nkp + 1);
      forest_commit(h, F, nullptr);
      make_private(h);
    } catch (...) {
      delete h;
      throw;
    }
    if (root32) memcpy(root32, h->root, 32);
    *out = h;
  })
}

int kh_trie_apply(kh_trie* h, const uint8_t* d_up_keys, const uint8_t* d_up_vals, const uint64_t* d_up_voff,
                  uint64_t nup, const uint8_t* d_del_keys, uint64_t ndel, uint32_t klen, uint32_t flags,
                  uint8_t root32[32], kh_stats* stats) {
  if (!h || h->forest) return set_err(KH_EINVAL, "null handle or a forest (use kh_forest_apply)");
  HANDLE_LOCK(h);
  API_TRY({
    HIPCHK(hipSetDevice(h->c->dev));
    check_flags(h, flags);
    FCommit F;
    F.up_keys = d_up_keys;
    F.up_vals = d_up_vals;
    F.up_voff = d_up_voff;
    F.nup = nup;
    F.del_keys = d_del_keys;
    F.ndel = ndel;
    F.klen = klen;
    forest_commit(h, F, stats);
    if (root32) memcpy(root32, h->root, 32);
  })
}

// host batch -> the context's staging buffers (keys of both kinds share in_keys)
static FCommit stage_commit(kh_ctx* c, const uint32_t* up_trie, const uint8_t* up_keys, const uint8_t* up_vals,
                            const uint64_t* up_voff, uint64_t nup, const uint32_t* del_trie, const uint8_t* del_keys,
                            uint64_t ndel, uint32_t klen) {
  const uint64_t v0 = nup ? up_voff[0] : 0, vb = nup ? up_voff[nup] - v0 : 0;
  HostPack P;
  const uint64_t ouk = P.add(up_keys, nup * klen), odk = P.add(del_keys, ndel * klen);
  const uint64_t ov = P.add(nup ? up_vals + v0 : nullptr, vb + (nup ? 0 : 0));
  const uint64_t oo = P.add(up_voff, nup ? (nup + 1) * 8 : 0, v0);
  const uint64_t out = P.add(up_trie, up_trie ? nup * 4 : 0), odt = P.add(del_trie, del_trie ? ndel * 4 : 0);
  P.total += 64;  // (slack past the values: 8-byte word reads)
  uint8_t* b = P.send(c, c->st);
  FCommit F;
  F.up_trie = up_trie ? (const uint32_t*)(b + out) : nullptr;
  F.up_keys = b + ouk;
  F.up_vals = b + ov;
  F.up_voff = (const uint64_t*)(b + oo);
  F.nup = nup;
  F.del_trie = del_trie ? (const uint32_t*)(b + odt) : nullptr;
  F.del_keys = b + odk;
  F.ndel = ndel;
  F.klen = klen;
  return F;
}

int kh_trie_apply_host(kh_trie* h, const uint8_t* up_keys, const uint8_t* up_vals, const uint64_t* up_voff,
                       uint64_t nup, const uint8_t* del_keys, uint64_t ndel, uint32_t klen, uint32_t flags,
                       uint8_t root32[32], kh_stats* stats) {
  if (!h || h->forest) return set_err(KH_EINVAL, "null handle or a forest (use kh_forest_apply_host)");
  API_TRY({
    HANDLE_LOCK(h);
    HIPCHK(hipSetDevice(h->c->dev));
    check_flags(h, flags);
    FCommit F = stage_commit(h->c, nullptr, up_keys, up_vals, up_voff, nup, nullptr, del_keys, ndel, klen);
    forest_commit(h, F, stats);
    if (root32) memcpy(root32, h->root, 32);
  })
}

int kh_forest_open(kh_ctx* c, uint32_t flags, kh_trie** out) {
  if (!out) return set_err(KH_EINVAL, "null handle");
  API_TRY({
    const bool host = !c;
    if (!c) c = shared_ctx(current_device());  // the context the *_host entry points use
    std::unique_ptr<kh_trie> h(trie_new(c, flags, true));
    if (host) make_private(h.get());
    *out = h.release();
  })
}

static int forest_out(kh_trie* f, uint32_t* h_tries, uint8_t* h_roots32, uint64_t cap, uint64_t* n_tries) {
  const uint64_t nt = f->tries.size();
  if (n_tries) *n_tries = nt;
  if (nt > cap || (nt && (!h_tries || !h_roots32))) return set_err(KH_ENOSPC, "trie output too small");
  if (nt) {
    memcpy(h_tries, f->tries.data(), nt * 4);
    memcpy(h_roots32, f->roots.data(), nt * 32);
  }
  return KH_OK;
}

int kh_forest_apply(kh_trie* f, const uint32_t* d_up_trie, const uint8_t* d_up_keys, const uint8_t* d_up_vals,
                    const uint64_t* d_up_voff, uint64_t nup, const uint32_t* d_del_trie, const uint8_t* d_del_keys,
                    uint64_t ndel, uint32_t klen, uint32_t* h_tries, uint8_t* h_roots32, uint64_t cap,
                    uint64_t* n_tries, kh_stats* stats) {
  if (!f || !f->forest) return set_err(KH_EINVAL, "null handle or not a forest");
  HANDLE_LOCK(f);
  API_TRY({
    HIPCHK(hipSetDevice(f->c->dev));
    FCommit F;
    F.up_trie = d_up_trie;
    F.up_keys = d_up_keys;
    F.up_vals = d_up_vals;
    F.up_voff = d_up_voff;
    F.nup = nup;
    F.del_trie = d_del_trie;
    F.del_keys = d_del_keys;
    F.ndel = ndel;
    F.klen = klen;
    forest_commit(f, F, stats);
    return forest_out(f, h_tries, h_roots32, cap, n_tries);
  })
}

int kh_forest_apply_host(kh_trie* f, const uint32_t* up_trie, const uint8_t* up_keys, const uint8_t* up_vals,
                         const uint64_t* up_voff, uint64_t nup, const uint32_t* del_trie, const uint8_t* del_keys,
                         uint64_t ndel, uint32_t klen, uint32_t* h_tries, uint8_t* h_roots32, uint64_t cap,
                         uint64_t* n_tries, kh_stats* stats) {
  if (!f || !f->forest) return set_err(KH_EINVAL, "null handle or not a forest");
  if ((nup && !up_trie) || (ndel && !del_trie)) return set_err(KH_EINVAL, "forest ops need trie ids");
  API_TRY({
    HANDLE_LOCK(f);
    HIPCHK(hipSetDevice(f->c->dev));
    FCommit F = stage_commit(f->c, up_trie, up_keys, up_vals, up_voff, nup, del_trie, del_keys, ndel, klen);
    forest_commit(f, F, stats);
    return forest_out(f, h_tries, h_roots32, cap, n_tries);
  })
}

int kh_forest_last_roots(kh_trie* f, uint32_t* h_tries, uint8_t* h_roots32, uint64_t cap, uint64_t* n_tries) {
  if (!f) return set_err(KH_EINVAL, "null handle");
  HANDLE_LOCK(f);
  API_TRY({ return forest_out(f, h_tries, h_roots32, cap, n_tries); })
}

int kh_trie_savepoint(kh_trie* h, uint32_t* depth) {
  if (!h) return set_err(KH_EINVAL, "null handle");
  HANDLE_LOCK(h);
  API_TRY({
    HIPCHK(hipSetDevice(h->c->dev));
    trie_savepoint(h);
    if (depth) *depth = (uint32_t)h->sps.size();
  })
}
int kh_trie_rollback(kh_trie* h) {
  if (!h) return set_err(KH_EINVAL, "null handle");
  API_TRY({
    HANDLE_LOCK(h);
    HIPCHK(hipSetDevice(h->c->dev));
    trie_rollback(h);
  })
}
int kh_trie_release(kh_trie* h) {
  if (!h) return set_err(KH_EINVAL, "null handle");
  HANDLE_LOCK(h);
  API_TRY({
    HIPCHK(hipSetDevice(h->c->dev));
    trie_release(h);
  })
}
int kh_trie_savepoint_depth(const kh_trie* h, uint32_t* depth) {
  if (!h || !depth) return set_err(KH_EINVAL, "null handle or output");
  HANDLE_LOCK(h);
  *depth = (uint32_t)h->sps.size();
  return KH_OK;
}

int kh_trie_root_of(kh_trie* h, const uint8_t* d_up_keys, const uint8_t* d_up_vals, const uint64_t* d_up_voff,
                    uint64_t nup, const uint8_t* d_del_keys, uint64_t ndel, uint32_t klen, uint32_t flags,
                    uint8_t root32[32], kh_stats* stats) {
  if (!h || h->forest) return set_err(KH_EINVAL, "null handle or a forest");
  HANDLE_LOCK(h);
  API_TRY({
    HIPCHK(hipSetDevice(h->c->dev));
    check_flags(h, flags);
    FCommit F;
    F.up_keys = d_up_keys;
    F.up_vals = d_up_vals;
    F.up_voff = d_up_voff;
    F.nup = nup;
    F.del_keys = d_del_keys;
    F.ndel = ndel;
    F.klen = klen;
    Txn txn(h, nullptr);
    forest_commit(h, F, stats);
    if (root32) memcpy(root32, h->root, 32);
    txn.rollback();
  })
}
int kh_trie_root_of_host(kh_trie* h, const uint8_t* up_keys, const uint8_t* up_vals, const uint64_t* up_voff,
                         uint64_t nup, const uint8_t* del_keys, uint64_t ndel, uint32_t klen, uint32_t flags,
                         uint8_t root32[32], kh_stats* stats) {
  if (!h || h->forest) return set_err(KH_EINVAL, "null handle or a forest");
  API_TRY({
    HANDLE_LOCK(h);
    HIPCHK(hipSetDevice(h->c->dev));
    check_flags(h, flags);
    FCommit F = stage_commit(h->c, nullptr, up_keys, up_vals, up_voff, nup, nullptr, del_keys, ndel, klen);
    Txn txn(h, nullptr);
    forest_commit(h, F, stats);
    if (root32) memcpy(root32, h->root, 32);
    txn.rollback();
  })
}

int kh_trie_copy(kh_trie* h, kh_trie** out) {
  if (!h || !out) return set_err(KH_EINVAL, "null handle");
  API_TRY({
    HANDLE_LOCK(h);
    HIPCHK(hipSetDevice(h->c->dev));
    *out = trie_copy(h);
  })
}

// The storage phase of a block runs on a second context of the device (its own streams and
// workspaces) on a host thread of its own, beside the account phase: the account keys are
// hashed, sorted and descended, and their elements gathered, while the storage tries commit;
// the account values are read only after the storage roots are injected into them
// (FCommit::before_values / vals_ready).
struct CtxSwap {  // a handle's commits on another context of the same device, for a scope
  kh_trie* h;
  kh_ctx* old;
  CtxSwap(kh_trie* t, kh_ctx* x) : h(t), old(t->c) { t->c = x; }
  ~CtxSwap() { h->c = old; }
};
int kh_block_commit(kh_trie* state, kh_trie* storage, const uint32_t* d_s_up_trie, const uint8_t* d_s_up_keys,
                    const uint8_t* d_s_up_vals, const uint64_t* d_s_up_voff, uint64_t ns_up,
                    const uint32_t* d_s_del_trie, const uint8_t* d_s_del_keys, uint64_t ns_del, uint32_t s_klen,
                    const uint8_t* d_a_up_keys, uint8_t* d_a_up_vals, const uint64_t* d_a_up_voff,
                    const uint32_t* d_a_up_trie, uint64_t na_up, const uint8_t* d_a_del_keys, uint64_t na_del,
                    uint32_t a_klen, uint8_t state_root32[32], kh_stats* stats) {
  if (!state || state->forest || !storage || !storage->forest) return set_err(KH_EINVAL, "need a state trie and a forest");
  if (state->home->dev != storage->home->dev) return set_err(KH_EINVAL, "state trie and forest on different devices");
  PairLock pl(state->lk, storage->lk);
  API_TRY({
    kh_ctx* c = state->c;
    HIPCHK(hipSetDevice(c->dev));
    hipStream_t st = c->st;
    kh_stats sst{}, ast{};
    // all or nothing: a refusal in either phase (or a device failure) rolls both handles back
    // to the parent version (Ledger.scala:237-271 discards the world state of a failed attempt)
    Txn txn(storage, state);
    // 1. every storage trie of the block (BlockWorldState.scala:243-252 -> TrieStorage.flush)
    FCommit S;
    S.up_trie = d_s_up_trie;
    S.up_keys = d_s_up_keys;
    S.up_vals = d_s_up_vals;
    S.up_voff = d_s_up_voff;
    S.nup = ns_up;
    S.del_trie = d_s_del_trie;
    S.del_keys = d_s_del_keys;
    S.ndel = ns_del;
    S.klen = s_klen;
    // 3. the accounts (TrieAccounts.flush, TrieAccounts.scala:22-28)
    FCommit A;
    A.up_keys = d_a_up_keys;
    A.up_vals = d_a_up_vals;
    A.up_voff = d_a_up_voff;
    A.nup = na_up;
    A.del_keys = d_a_del_keys;
    A.ndel = na_del;
    A.klen = a_klen;
    A.chk_msg = "an account upsert with a storage trie is not an account body";
    if (c->pack_for_block) S.inputs_ready = A.inputs_ready = c->pack_ev;  // (host inputs: one DMA on c->st)
    // the injection's error word (never cleared: a failing call writes its own token into it)
    if (!c->ws_inject.p) {
      c->ws_inject.ensure(64);
      HIPCHK(hipMemsetAsync(c->ws_inject.p, 0, 64, st));
      HIPCHK(hipStreamSynchronize(st));
    }
    unsigned long long* err = (unsigned long long*)c->ws_inject.p;
    const unsigned long long tok = ++c->inject_tok;
    // 2. account.withStateRoot: the new storage roots into the account bodies (the forest's trie
    // list and roots are still on the device: its commit's tbuf)
    auto inject = [&](hipStream_t s, uint32_t nt) {  // nt: the storage commit's touched tries
      if (!(nt && na_up && d_a_up_trie && storage->d_tries)) return false;  // (set by this call's storage commit)
      hipLaunchKernelGGL(k_inject_roots, GRID(na_up, BS), dim3(BS), 0, s, d_a_up_vals, d_a_up_voff, d_a_up_trie,
                         na_up, (const uint32_t*)storage->d_tries, nt, (const uint64_t*)storage->d_roots, err, tok);
      LAUNCH_CHECK();
      return true;
    };
    const bool overlap = (ns_up + ns_del) && (na_up + na_del);
    if (!overlap) {
      forest_commit(storage, S, &sst);
      if (inject(st, (uint32_t)storage->tries.size())) {  // (read back with the account commit's first sync, before it changes anything)
        A.chk = err;
        A.chk_tok = tok;
      }
      forest_commit(state, A, &ast);
    } else {
      // the storage phase on the forest's own context (private handles), or on a second context
      // of the state trie's
      const bool own = storage->c != c;
      if (!own && !c->bsub) c->bsub = ctx_new(c->dev);
      if (!c->bev) HIPCHK(hipEventCreateWithFlags(&c->bev, hipEventDisableTiming));
      kh_ctx* aux = own ? storage->c : c->bsub;
      std::mutex mu;
      std::condition_variable cv;
      bool done = false, injected = false;
      std::exception_ptr serr, aerr;
      if (!c->bworker) c->bworker.reset(new Worker());
      // the injection as soon as the storage roots are on the device (FCommit::after_roots),
      // before the storage phase's records and anchor map; once, and at the end if the phase
      // had no element build
      auto inject_once = [&](hipStream_t s, uint32_t nt) {
        if (injected) return;
        inject(s, nt);
        HIPCHK(hipEventRecord(c->bev, s));
        {
          std::lock_guard<std::mutex> lk(mu);
          injected = true;
        }
        cv.notify_all();
      };
      S.after_roots = inject_once;
      c->bworker->post([&] {
        try {
          HIPCHK(hipSetDevice(c->dev));
          CtxSwap sw(storage, aux);
          forest_commit(storage, S, &sst);
          inject_once(aux->st, (uint32_t)storage->tries.size());
        } catch (...) {
          serr = std::current_exception();
        }
        {
          std::lock_guard<std::mutex> lk(mu);
          done = true;
        }
        cv.notify_all();
        (void)hipStreamSynchronize(aux->st);  // nothing of the phase is left in flight
      });
      A.chk = err;  // (only an injection that failed writes this call's token)
      A.chk_tok = tok;
      A.vals_ready = c->bev;
      A.late = d_a_up_trie;  // the bodies that get a storage root; the rest are hashed before it
      A.late_ready = [&] {  // the injection already DONE on the device (merely enqueued, the storage
                            // phase's queue may still hold ~0.2 ms of work: the other leaves go first)
        std::lock_guard<std::mutex> lk(mu);
        return injected && hipEventQuery(c->bev) == hipSuccess;
      };
      A.before_values = [&] {
        std::unique_lock<std::mutex> lk(mu);
        cv.wait(lk, [&] { return injected || done; });
        if (!injected) throw KhError{KH_EINTERNAL, "the block's storage phase failed"};
      };
      try {
        forest_commit(state, A, &ast);
      } catch (...) {
        aerr = std::current_exception();
      }
      c->bworker->join();
      if (serr) std::rethrow_exception(serr);
      if (aerr) std::rethrow_exception(aerr);
    }
    // all or nothing, also for the lazy tails (records, anchor maps) still in flight: a failure
    // there rolls both handles back (~Txn) instead of surfacing on a later call
    trie_settle(storage);
    trie_settle(state);
    txn.release();
    memcpy(state_root32, state->root, 32);
    if (stats) {
      *stats = ast;
      stats->n_inputs = ast.n_inputs + sst.n_inputs;
      stats->n_node_hashes = ast.n_node_hashes + sst.n_node_hashes;
      stats->n_node_perms = ast.n_node_perms + sst.n_node_perms;
      stats->n_key_perms = ast.n_key_perms + sst.n_key_perms;
      stats->n_branches = ast.n_branches + sst.n_branches;
      stats->t_total_ms = ast.t_total_ms + sst.t_total_ms;
    }
  })
}

// kh_block_commit from host arrays (the JVM caller): the block's whole dirty set staged
// in one buffer, then the device variant
int kh_block_commit_host(kh_trie* state, kh_trie* storage, const uint32_t* s_up_trie, const uint8_t* s_up_keys,
                         const uint8_t* s_up_vals, const uint64_t* s_up_voff, uint64_t ns_up,
                         const uint32_t* s_del_trie, const uint8_t* s_del_keys, uint64_t ns_del, uint32_t s_klen,
                         const uint8_t* a_up_keys, const uint8_t* a_up_vals, const uint64_t* a_up_voff,
                         const uint32_t* a_up_trie, uint64_t na_up, const uint8_t* a_del_keys, uint64_t na_del,
                         uint32_t a_klen, uint8_t state_root32[32], kh_stats* stats) {
  if (!state || !storage) return set_err(KH_EINVAL, "need a state trie and a forest");
  if ((ns_up && (!s_up_trie || !s_up_voff)) || (ns_del && !s_del_trie) || (na_up && !a_up_voff))
    return set_err(KH_EINVAL, "null input");
  kh_ctx* c = state->c;
  PairLock pl(state->lk, storage->lk);
  int rc = KH_OK;
  try {
    HIPCHK(hipSetDevice(c->dev));
    const uint64_t sv0 = ns_up ? s_up_voff[0] : 0, svb = ns_up ? s_up_voff[ns_up] - sv0 : 0;
    const uint64_t av0 = na_up ? a_up_voff[0] : 0, avb = na_up ? a_up_voff[na_up] - av0 : 0;
    HostPack P;
    const uint64_t o_st = P.add(s_up_trie, ns_up * 4), o_sk = P.add(s_up_keys, ns_up * s_klen);
    const uint64_t o_sv = P.add(s_up_vals ? s_up_vals + sv0 : nullptr, svb), o_so = P.add(s_up_voff, ns_up ? (ns_up + 1) * 8 : 0, sv0);
    const uint64_t o_sdt = P.add(s_del_trie, ns_del * 4), o_sdk = P.add(s_del_keys, ns_del * s_klen);
    const uint64_t o_ak = P.add(a_up_keys, na_up * a_klen), o_av = P.add(a_up_vals ? a_up_vals + av0 : nullptr, avb);
    const uint64_t o_ao = P.add(a_up_voff, na_up ? (na_up + 1) * 8 : 0, av0);
    const uint64_t o_at = P.add(a_up_trie, a_up_trie ? na_up * 4 : 0), o_adk = P.add(a_del_keys, na_del * a_klen);
    P.total += 64;
    uint8_t* base = P.send(c, c->st);  // (the storage phase may run on another stream: pack_for_block)
    c->pack_for_block = true;
    uint32_t* st_ = (uint32_t*)(base + o_st);
    uint8_t* sk = base + o_sk;
    uint8_t* sv = base + o_sv;
    uint64_t* so = (uint64_t*)(base + o_so);
    uint32_t* sdt = (uint32_t*)(base + o_sdt);
    uint8_t* sdk = base + o_sdk;
    uint8_t* ak = base + o_ak;
    uint8_t* av = base + o_av;
    uint64_t* ao = (uint64_t*)(base + o_ao);
    uint32_t* at = (uint32_t*)(base + o_at);
    uint8_t* adk = base + o_adk;
    rc = kh_block_commit(state, storage, st_, sk, sv, so, ns_up, sdt, sdk, ns_del, s_klen, ak, av, ao,
                         a_up_trie ? at : nullptr, na_up, adk, na_del, a_klen, state_root32, stats);
    c->pack_for_block = false;
  } catch (KhError& e) {
    return set_err(e.code, e.msg);
  } catch (std::exception& e) {
    return set_err(KH_EINTERNAL, e.what());
  }
  return rc;
}

int kh_trie_emit_nodes(kh_trie* h, uint8_t* hashes32, uint64_t node_cap, uint8_t* rlp, uint64_t rlp_cap,
                       uint64_t* off, uint64_t* n_nodes, uint64_t* rlp_len) {
  if (!h || !n_nodes || !rlp_len) return set_err(KH_EINVAL, "null handle or size outputs");
  HANDLE_LOCK(h);
  API_TRY({
    if (!(h->flags & KH_EMIT_NODES)) throw KhError{KH_EINVAL, "trie opened without KH_EMIT_NODES"};
    HIPCHK(hipSetDevice(h->c->dev));
    if (!h->em_valid) {
      *n_nodes = *rlp_len = 0;
      if (off) off[0] = 0;
      return KH_OK;
    }
    return emit_to_host(h->c, h->em, h->em_n, h->em_bytes, hashes32, node_cap, rlp, rlp_cap, off, n_nodes, rlp_len);
  })
}

// ---- batched get (MerklePatriciaTrie.get, MerklePatriciaTrie.scala:90-147)
__global__ void __launch_bounds__(BS) k_get_find(AMap M, Recs R, const uint64_t* K, const uint32_t* trie, uint64_t n,
                                                 uint32_t* rec, uint64_t* len) {
  const uint64_t o = (uint64_t)blockIdx.x * BS + threadIdx.x;
  if (o >= n) return;
  const uint32_t r = forest_get(M, R, trie ? trie[o] : 0u, K + 4 * o);
  rec[o] = r;
  len[o] = r == NONE ? 0 : R.rvl[r];
}
// value bytes into the packed output (one thread per query; values are short)
__global__ void __launch_bounds__(BS) k_get_copy(Recs R, const uint8_t* heap, const uint32_t* rec, const uint64_t* voff,
                                                 uint64_t n, uint8_t* out, uint8_t* found) {
  const uint64_t o = (uint64_t)blockIdx.x * BS + threadIdx.x;
  if (o >= n) return;
  const uint32_t r = rec[o];
  found[o] = r != NONE;
  if (r == NONE) return;
  const uint8_t* src = heap + R.rvo[r];
  uint8_t* dst = out + voff[o];
  for (uint32_t b = 0, L = R.rvl[r]; b < L; ++b) dst[b] = src[b];
}

// n queries (device buffers): the keys (the trie's key encoder applied, as in a commit),
// their trie ids (forests; NULL = trie 0), then the found flags, the packed values and
// their offsets.  Returns KH_ENOSPC (writing only *val_bytes) when val_cap is too small.
static int trie_get(kh_trie* h, const uint32_t* d_trie, const uint8_t* d_keys, uint32_t klen, uint64_t n,
                    uint8_t* d_vals, uint64_t val_cap, uint64_t* d_voff, uint8_t* d_found, uint64_t* val_bytes) {
  kh_ctx* c = h->c;
  hipStream_t st = c->st;
  if (h->forest && n && !d_trie) throw KhError{KH_EINVAL, "forest queries need trie ids"};
  if (!(h->flags & KH_HASH_KEYS) && klen != 32) throw KhError{KH_EINVAL, "keys must be 32 bytes unless KH_HASH_KEYS"};
  if (klen == 0 || klen > 4096) throw KhError{KH_EINVAL, "bad key length"};
  if (n >= (1ULL << 31)) throw KhError{KH_EINVAL, "too many queries"};
  h->gbuf.ensure(carve_size({n * 32 + 64, n * 4, (n + 1) * 8, scan_scratch_bytes(n + 1, 8), 64}));
  Carver cv{(char*)h->gbuf.p, 0, h->gbuf.cap};
  uint64_t* K = cv.take<uint64_t>(n * 4 + 8);
  uint32_t* rec = cv.take<uint32_t>(n);
  uint64_t* len = cv.take<uint64_t>(n + 1);
  char* scr = cv.take<char>(scan_scratch_bytes(n + 1, 8));
  uint64_t* tot = cv.take<uint64_t>(8);
  if (n) {
    if (h->flags & KH_HASH_KEYS) {
      if (klen <= 135)
        hipLaunchKernelGGL(k_hash_keys<true>, GRID(n, BS), dim3(BS), 0, st, d_keys, klen, n, K);
      else
        hipLaunchKernelGGL(k_hash_keys<false>, GRID(n, BS), dim3(BS), 0, st, d_keys, klen, n, K);
      LAUNCH_CHECK();
    } else {
      HIPCHK(hipMemcpyAsync(K, d_keys, n * 32, hipMemcpyDeviceToDevice, st));
    }
    if (h->rn && h->mcap) {
      hipLaunchKernelGGL(k_get_find, GRID(n, BS), dim3(BS), 0, st, map_of(h), recs_of(h), (const uint64_t*)K, d_trie,
                         n, rec, len);
      LAUNCH_CHECK();
    } else {  // an empty trie or forest
      HIPCHK(hipMemsetAsync(rec, 0xFF, n * 4, st));
      HIPCHK(hipMemsetAsync(len, 0, n * 8, st));
    }
    scan_exclusive<uint64_t>(len, d_voff, n, tot, scr, st);
    HIPCHK(hipMemcpyAsync(d_voff + n, tot, 8, hipMemcpyDeviceToDevice, st));
    HIPCHK(hipMemcpyAsync(c->h_pinned, tot, 8, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
  } else {
    HIPCHK(hipMemsetAsync(d_voff, 0, 8, st));
    HIPCHK(hipStreamSynchronize(st));
    c->h_pinned[0] = 0;
  }
  const uint64_t total = c->h_pinned[0];
  if (val_bytes) *val_bytes = total;
  if (total > val_cap) return set_err(KH_ENOSPC, "value output too small (*val_bytes holds the size needed)");
  if (n) {
    hipLaunchKernelGGL(k_get_copy, GRID(n, BS), dim3(BS), 0, st, recs_of(h), (const uint8_t*)h->heap.p,
                       (const uint32_t*)rec, (const uint64_t*)d_voff, n, d_vals, d_found);
    LAUNCH_CHECK();
  }
  HIPCHK(hipStreamSynchronize(st));
  return KH_OK;
}

int kh_trie_get(kh_trie* h, const uint32_t* d_trie, const uint8_t* d_keys, uint32_t klen, uint64_t n, uint8_t* d_vals,
                uint64_t val_cap, uint64_t* d_voff, uint8_t* d_found, uint64_t* val_bytes) {
  if (!h) return set_err(KH_EINVAL, "null handle");
  if (!d_voff || (n && (!d_keys || !d_found))) return set_err(KH_EINVAL, "null buffer");
  HANDLE_LOCK(h);
  API_TRY({
    HIPCHK(hipSetDevice(h->c->dev));
    return trie_get(h, d_trie, d_keys, klen, n, d_vals, val_cap, d_voff, d_found, val_bytes);
  })
}

int kh_trie_get_host(kh_trie* h, const uint32_t* trie, const uint8_t* keys, uint32_t klen, uint64_t n, uint8_t* vals,
                     uint64_t val_cap, uint64_t* voff, uint8_t* found, uint64_t* val_bytes) {
  if (!h) return set_err(KH_EINVAL, "null handle");
  if (!voff || (n && (!keys || !found))) return set_err(KH_EINVAL, "null buffer");
  API_TRY({
    HANDLE_LOCK(h);
    kh_ctx* c = h->c;
    HIPCHK(hipSetDevice(c->dev));
    hipStream_t st = c->st;
    // staging: keys and trie ids in, found flags, offsets and values out
    c->in_keys.ensure(carve_size({n * klen + 64, trie ? n * 4 : 0}));
    Carver ck{(char*)c->in_keys.p, 0, c->in_keys.cap};
    uint8_t* dk = ck.take<uint8_t>(n * klen + 64);
    uint32_t* dt = trie ? ck.take<uint32_t>(n) : nullptr;
    c->in_voff.ensure((n + 1) * 8 + 64);
    c->out_emit.ensure(carve_size({n + 64, val_cap + 64}));
    Carver co{(char*)c->out_emit.p, 0, c->out_emit.cap};
    uint8_t* df = co.take<uint8_t>(n + 64);
    uint8_t* dv = co.take<uint8_t>(val_cap + 64);
    if (n) HIPCHK(hipMemcpyAsync(dk, keys, n * klen, hipMemcpyHostToDevice, st));
    if (dt) HIPCHK(hipMemcpyAsync(dt, trie, n * 4, hipMemcpyHostToDevice, st));
    const int rc = trie_get(h, dt, dk, klen, n, dv, val_cap, (uint64_t*)c->in_voff.p, df, val_bytes);
    if (rc != KH_OK) return rc;
    HIPCHK(hipMemcpyAsync(voff, c->in_voff.p, (n + 1) * 8, hipMemcpyDeviceToHost, st));
    if (n) HIPCHK(hipMemcpyAsync(found, df, n, hipMemcpyDeviceToHost, st));
    const uint64_t tot = val_bytes ? *val_bytes : 0;
    HIPCHK(hipStreamSynchronize(st));
    const uint64_t total = n ? voff[n] : tot;
    if (total) HIPCHK(hipMemcpyAsync(vals, dv, total, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
  })
}

int kh_trie_compact(kh_trie* h, kh_trie_usage_t* before) {
  if (!h) return set_err(KH_EINVAL, "null handle");
  API_TRY({
    HANDLE_LOCK(h);
    HIPCHK(hipSetDevice(h->c->dev));
    trie_compact(h, before);
  })
}

int kh_trie_usage(kh_trie* h, kh_trie_usage_t* u) {
  if (!h || !u) return set_err(KH_EINVAL, "null handle");
  API_TRY({
    HANDLE_LOCK(h);
    HIPCHK(hipSetDevice(h->c->dev));
    trie_usage(h, u);
  })
}

int kh_trie_size(const kh_trie* h, uint64_t* n) {
  if (!h || !n) return set_err(KH_EINVAL, "null handle");
  HANDLE_LOCK(h);
  *n = h->nleaves;
  return KH_OK;
}

int kh_trie_free(kh_trie* h) {
  if (!h) return KH_OK;
  API_TRY({
    {  // (a handle's own mutex goes with it: released before the delete)
      HANDLE_LOCK(h);
      (void)hipSetDevice(h->c->dev);
      (void)hipStreamSynchronize(h->c->st);
      (void)hipStreamSynchronize(h->c->st2);
    }
    delete h;  // every DevBuf releases its HBM; a private context is destroyed with it
  })
}

}  // extern "C"

// multi-GPU root over RCCL in one process (kh_trie_root_sharded)
#include "sharded.h"
