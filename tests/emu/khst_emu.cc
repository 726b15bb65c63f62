// TEST INFRASTRUCTURE ONLY — host replay of the device pipeline.
//
// Compiles khipu_amd/csrc/trie_ops.h (the per-thread bodies of the HIP kernels)
// with g++ and drives them with plain loops, std::stable_sort in place of the
// radix sort and std::partial_sum in place of the device scan.  It lets the CPU
// test suite check the topology / RLP / Keccak logic of the GPU path against the
// oracle without a GPU.  It is never linked into libkhst.so and the product
// never calls it; the GPU parity tests (tests/test_gpu_parity.py) exercise the
// real kernels.
#include <algorithm>
#include <array>
#include <random>
#include <cstring>
#include <numeric>
#include <string>
#include <vector>

#include "../../khipu_amd/csrc/nodedata.h"
#include "../../khipu_amd/csrc/keyorder.h"
#include "../../khipu_amd/csrc/synth.h"
#include "../../khipu_amd/csrc/keccak_xlane.h"

using namespace khst;

// The device's tile-local topology (khst.hip k_topo_tile, then k_ansv_list / k_chain_list
// after the whole-array pyramid P) replayed tile by tile with tiles of `tile` boundaries.  With
// the device's tile size the tile's 64-boundary minima must be the pyramid's first level (the
// device's tile kernel writes that level; k_pyramid starts above it): g_pyr1_bad counts misses.
static uint64_t g_pyr1_bad = 0;
static void topo_tiles(const Topo& T, const Pyr& P, uint64_t nb, uint32_t tile) {
  std::vector<uint32_t> alist, clist;
  std::vector<uint8_t> su(TOPO_TILE + 16), sl1(64 + 16);
  std::vector<int16_t> lpse(TOPO_TILE);
  std::vector<uint8_t> lnext(TOPO_TILE), lrin(TOPO_TILE);
  for (uint64_t t0 = 0; t0 < nb; t0 += tile) {
    const uint32_t tn = (uint32_t)(nb - t0 < tile ? nb - t0 : tile);
    std::fill(su.begin(), su.end(), (uint8_t)0x7F);
    memcpy(su.data(), T.u + t0, tn);
    std::fill(lnext.begin(), lnext.end(), (uint8_t)0);
    std::fill(lrin.begin(), lrin.end(), (uint8_t)0x5A);  // (set by phase 1 wherever phase 2 reads it)
    for (uint32_t w = 0; w < 64; ++w) {
      uint32_t mn = 0x7F;
      for (uint32_t q = 0; q < 64 && 64 * w + q < TOPO_TILE; ++q) mn = std::min(mn, (uint32_t)su[64 * w + q]);
      sl1[w] = (uint8_t)mn;
      if (tile == TOPO_TILE && P.nl > 1 && 64 * w < tn && P.lv[1][t0 / 64 + w] != (uint8_t)mn) ++g_pyr1_bad;
    }
    const TilePyr L{su.data(), sl1.data(), tn, (tn + 63) / 64};
    for (uint32_t i = 0; i < tn; ++i)
      if (op_tile_ansv(T, L, t0, i, lpse.data(), lnext.data(), lrin.data())) alist.push_back((uint32_t)(t0 + i));
    for (uint32_t i = 0; i < tn; ++i) {
      uint32_t isr = 0;
      if (op_tile_chain(T, L, t0, i, lpse.data(), lnext.data(), lrin.data(), &isr)) clist.push_back((uint32_t)(t0 + i));
      if (T.rep_bits && isr) T.rep_bits[(t0 + i) >> 5] |= 1u << ((t0 + i) & 31);  // (the device's per-wave ballot words)
    }
  }
  for (uint32_t b : alist) op_ansv(T, P, b);
  for (uint32_t b : clist) op_chain(T, b);
}

// which form of the early leaf kernel the replay runs: 0 / 1 = op_leaf_in3 with the
// loosest / the lane's own wave bounds (every dword masked / every dword classified)
static int g_leaf_mode = 0;
// 0: link slots + the copy pass (op_leaf_link / op_leaf_move: the device's segmented
// builds); 2: leaf positions (the device's unsegmented builds): no leaf child records, the
// branches read each leaf child's stash at its sorted position, on alternate branches
// straight from the stash (op_branch_stream) and through the records a small level writes
// first (op_leaf_children)
static int g_link_mode = 0;
// a corrupt boundary value injected into u[g_inject_j] (the r5y fault: stale bytes): 1 before
// the leaves' parent-depth scatter (value 200), 2 before the branch records (value 70), 3 the
// scatter with value 1 under depth0 = 1 (below the first valid value 2)
static int g_inject = 0;
static uint64_t g_inject_j = 0;

// keys: n*32 (already keccak'd), vals/voff packed; seg nullable.
// Outputs per result r: hash (32 B), enc length, inline bytes (32 B).
// stats_out[0..5] = m, B, node hashes, node perms, inline nodes, extensions.
static int build_core(const uint8_t* keys, const uint8_t* vals, const uint64_t* voff, uint64_t n, const uint32_t* seg,
                      uint64_t nseg, uint32_t depth0, uint8_t* out_hash, uint32_t* out_len, uint8_t* out_inl,
                      uint64_t* stats_out) {
  const bool segmented = seg != nullptr;
  const uint64_t nres = segmented ? nseg : (depth0 == 1 ? 16 : 1);
  std::vector<uint64_t> res_hash(nres * 4, 0), res_inl(nres * 4, 0);
  std::vector<uint32_t> res_len(nres, 0);
  if (n == 0) {
    memset(out_len, 0, nres * 4);
    return 0;
  }
  // sort (stable, by segment then key bytes), keep the last duplicate
  std::vector<uint32_t> order(n);
  std::iota(order.begin(), order.end(), 0u);
  std::stable_sort(order.begin(), order.end(), [&](uint32_t a, uint32_t b) {
    if (segmented && seg[a] != seg[b]) return seg[a] < seg[b];
    return memcmp(keys + 32ull * a, keys + 32ull * b, 32) < 0;
  });
  std::vector<uint32_t> sidx;
  for (uint64_t i = 0; i < order.size(); ++i) {
    bool dup_next = i + 1 < order.size() && memcmp(keys + 32ull * order[i], keys + 32ull * order[i + 1], 32) == 0 &&
                    (!segmented || seg[order[i]] == seg[order[i + 1]]);
    if (!dup_next) sidx.push_back(order[i]);
  }

  const uint64_t m = sidx.size(), nb = m - 1;
  std::vector<uint64_t> skey(4 * m);
  std::vector<uint32_t> sseg(m);
  for (uint64_t i = 0; i < m; ++i) {
    memcpy(&skey[4 * i], keys + 32ull * sidx[i], 32);
    if (segmented) sseg[i] = seg[sidx[i]];
  }
  Topo T{};
  T.m = m;
  T.depth0 = depth0;
  T.segmented = segmented;
  T.skey = skey.data();
  T.sidx = sidx.data();
  T.sseg = sseg.data();
  T.vals = vals;
  T.voff = voff;
  std::vector<uint64_t> svoff(m);
  std::vector<uint32_t> svlen(m);
  T.svoff = svoff.data();
  T.svlen = svlen.data();
  for (uint64_t i = 0; i < m; ++i) op_val_gather(T, i);
  const uint64_t nbb = nb + 1;
  std::vector<uint8_t> glast(nbb, 1), gk(nbb, 0);
  std::vector<uint8_t> u(nbb), ord(nbb), br_depth(nbb), br_ext(nbb), br_pord(nbb), lf_pord(m);
  std::vector<int32_t> psv(nbb), nsv(nbb), pse(nbb);
  std::vector<uint32_t> rep(nbb), isrep(nbb), br_k(nbb, 0), br_cbase(nbb), br_parent(nbb), br_first(nbb),
      br_len(nbb), ex_len(nbb), lf_parent(m), lf_len(m);
  std::vector<int8_t> lf_pd(m);
  std::vector<uint64_t> br_aoff(nbb), lf_aoff(m);
  std::vector<unsigned long long> ctr(2 * CTR_N, 0);
  std::vector<uint32_t> hist(64, 0);
  T.u = u.data();
  T.psv = psv.data();
  T.nsv = nsv.data();
  T.pse = pse.data();
  T.rep = rep.data();
  T.ord = ord.data();
  T.isrep_bid = isrep.data();
  T.glast = glast.data();
  T.gk = gk.data();
  T.br_k = br_k.data();
  T.br_cbase = br_cbase.data();
  T.br_depth = br_depth.data();
  T.br_ext = br_ext.data();
  T.br_parent = br_parent.data();
  T.br_pord = br_pord.data();
  T.br_first = br_first.data();
  T.br_aoff = br_aoff.data();
  T.br_len = br_len.data();
  T.ex_len = ex_len.data();
  T.lf_parent = lf_parent.data();
  T.lf_pord = lf_pord.data();
  T.lf_pd = lf_pd.data();
  T.lf_aoff = lf_aoff.data();
  T.lf_len = lf_len.data();
  T.res_hash = res_hash.data();
  T.res_len = res_len.data();
  T.res_inl = res_inl.data();
  T.ctr = ctr.data();
  T.depth_hist = hist.data();
  uint64_t B = 0;
  const bool lpos = g_link_mode == 2 && !segmented;
  std::vector<uint32_t> br_end(nbb, 0);
  if (lpos) {
    T.br_end = br_end.data();
    T.lpos = 1;
  }
  std::vector<std::vector<uint8_t>> pyr;
  Pyr P{};
  // the representative flags as bits, as the device's early tile builds keep them (the branch ids
  // stay in key order here: the replay's levels list them by depth, no permutation); they live
  // for the whole build (the leaves resolve their parents through them)
  const uint64_t nw = (nb + 31) / 32 + 1;
  std::vector<uint32_t> rbits(nw, 0), rpref(nw + 1, 0);
  // unsegmented builds take the device's ck path: boundary values from the sorted first
  // key words (the input keys past them), before the sorted keys are used
  std::vector<uint64_t> kin(4 * n + 4);
  std::vector<uint32_t> sck(m + 1);
  memcpy(kin.data(), keys, 32 * n);
  T.kin = kin.data();
  if (!segmented) {
    for (uint64_t i = 0; i < m; ++i) sck[i] = (uint32_t)(bswap64(skey[4 * i]) >> 32);
    T.sck = sck.data();
    T.skey = nullptr;  // as on the device: no sorted keys on this path
  }
  if (nb > 0) {
    for (uint64_t b = 0; b < nb; ++b) op_lcp(T, b);
    P.lv[0] = T.u;
    P.sz[0] = nb;
    P.nl = 1;
    pyr.reserve(8);
    while (P.sz[P.nl - 1] > 64) {
      uint64_t nin = P.sz[P.nl - 1], nout = (nin + 63) / 64;
      pyr.emplace_back(nout);
      for (uint64_t i = 0; i < nout; ++i) op_min64(P.lv[P.nl - 1], nin, pyr.back().data(), i);
      P.lv[P.nl] = pyr.back().data();
      P.sz[P.nl] = nout;
      P.nl++;
    }
    T.rep_bits = rbits.data();
    T.rep_pref = rpref.data();
    g_pyr1_bad = 0;
    topo_tiles(T, P, nb, TOPO_TILE);  // (as on the device)
    if (ctr[CTR_ERR]) return -5;
    if (g_pyr1_bad) return -10;
    uint32_t run = 0;
    for (uint64_t w = 0; w < nw; ++w) {
      rpref[w] = run;
      run += (uint32_t)__builtin_popcount(rbits[w]);
    }
    B = run;
    if (g_inject == 2)  // the first representative boundary from g_inject_j on
      for (uint64_t b = g_inject_j; b < nb; ++b)
        if (u[b] && rep[b] == b) {
          u[b] = 70;
          break;
        }
    for (uint64_t b = 0; b < nb; ++b) {
      const uint32_t xf = op_branch_topo(T, P, nb, b);
      if (ctr[CTR_ERR] == ERR_LEAF_TOPO) return -9;  // (the device: KH_EINTERNAL at the topology's counter sync)
      if (u[b] != 0 && rep[b] == b) {
        uint32_t j = bid_of(T, b);
        hist[br_depth[j]]++;
        if (br_ext[j]) ctr[CTR_EXT]++;
        if (xf != (br_ext[j] ? 1u : 0u)) return -8;  // (the device counts extensions from the return value)
      }
    }
  }
  // plain builds replay the device's early-leaf path: parent depths scattered to input
  // order (k_pd_scatter), leaves hashed in input order (k_leaf_in), references stashed
  // per input and published after the topology
  std::vector<uint64_t> eref(4 * m + 4);
  std::vector<uint8_t> emeta(m + 1, 32);  // preset as on the device
  std::vector<uint64_t> pdinv(n + 1, PDINV_SKIP);
  uint64_t perms = 0, hashes = 0, inl = 0, longb = 0;
  T.lf_eref = eref.data();
  T.lf_emeta = emeta.data();
  T.pdinv = pdinv.data();
  std::vector<uint32_t> longlist(m + 1);
  T.longlist = lpos ? longlist.data() : nullptr;
  T.svoff = nullptr;  // as on the device: no sorted spans in early builds
  T.svlen = nullptr;
  if ((g_inject == 1 || g_inject == 3) && g_inject_j < nb) u[g_inject_j] = g_inject == 1 ? 200 : 1;
  for (uint64_t i = 0; i < m; ++i) op_pd_scatter(T, i);
  // the device reads whole 16-byte-aligned pairs around each span: replay on a copy of
  // the values at byte 8 of a 16-byte pair, with zero pairs either side (host memory is
  // not page-granular)
  std::vector<uint64_t> vbuf(voff[n] / 8 + 8, 0);
  uint8_t* vbase = (uint8_t*)(((uintptr_t)vbuf.data() + 15) & ~(uintptr_t)15);
  memcpy(vbase + 24, vals, voff[n]);
  T.vals = vbase + 24;
  // the keys likewise: the device kernel reads a shifted window of up to 3 keys past the
  // current one (edge lanes take clamped loads)
  std::vector<uint64_t> kbuf(4 * n + 16, 0);
  if (n) memcpy(kbuf.data(), T.kin, 32 * n);
  T.kin = kbuf.data();
  {
    // op_leaf_in3 with the loosest wave bounds (mode 0: every dword takes its masked form)
    // or the lane's own values (mode 1: every dword takes its classified form)
    auto wave = [](bool use, uint32_t e, uint32_t llo, uint32_t lhi) {
      if (g_leaf_mode == 0 || !use) return WaveBounds{0, 255, 0, 255};
      return WaveBounds{e, e, llo, lhi};
    };
    for (uint64_t j = 0; j < n + 3; ++j) {  // lanes past the end take part as on the device
      uint32_t in1 = 0, lb = 0;
      uint32_t p = op_leaf_in3(T, j, n, wave, &in1, &lb);
      perms += p;
      hashes += p ? 1 : 0;
      inl += in1;
      longb += lb;
    }
  }
  if (ctr[CTR_ERR] == ERR_LEAF_TOPO) return -9;  // (the device: KH_EINTERNAL at the leaves' counter sync)
  uint64_t C = 0;
  for (uint64_t j = 0; j < B; ++j) {
    br_cbase[j] = (uint32_t)C;
    C += br_k[j];
  }
  uint64_t lfb = 0;
  std::vector<uint64_t> cref(4 * C + 4);
  std::vector<uint16_t> cmeta(C + 1);
  T.cref = cref.data();
  T.cmeta = cmeta.data();
  auto bump = [&](uint64_t b) {
    uint64_t o = lfb;
    lfb += b;
    return o;
  };
  std::vector<uint64_t> dst(m + 1);
  T.lf_dst = dst.data();
  std::vector<uint32_t> cend(C + 1, 0);
  if (lpos) {  // only the long leaves' parents and arena slots
    T.lf_inline = inl ? 1 : 0;
    for (uint64_t q = 0; q < ctr[CTR_LONGN]; ++q) op_leaf_topo_early(T, longlist[q], bump);
  } else {  // the device's split publish: slots during the hashing, then the copy
    for (uint64_t i = 0; i < m; ++i) op_leaf_link(T, i);
    for (uint64_t i = 0; i < m; ++i) op_leaf_move(T, i, bump);
  }
  if (lfb != longb) return -7;  // the arena is sized by the early count
  std::vector<uint64_t> arena((lfb + 64) / 8 + 1), lmsg(LEAF_WORDS * m + 1), bmsg(BR_WORDS * B + 1),
      xmsg(EXT_WORDS * B + 1);
  T.lmsg = lmsg.data();
  T.lstride = m;
  T.bmsg = bmsg.data();
  T.xmsg = xmsg.data();
  // level order: branch ids bucketed by depth (ascending id inside a level)
  std::vector<uint32_t> lbv(65, 0), lorder;
  for (int d = 0; d < 64; ++d) {
    lbv[d] = (uint32_t)lorder.size();
    for (uint64_t j = 0; j < B; ++j)
      if (br_depth[j] == d) lorder.push_back((uint32_t)j);
  }
  lbv[64] = (uint32_t)lorder.size();
  T.lb = lbv.data();
  std::vector<uint8_t> br_dirty(B + 1, 1);
  T.arena = (uint8_t*)arena.data();
  if (lpos) T.cend = cend.data();  // (set after the leaf kernel, as on the device)
  for (uint64_t i = 0; i < m; ++i) {
    uint32_t in1 = 0;
    uint32_t p = op_leaf_long(T, i, &in1);
    perms += p;
    hashes += p ? 1 : 0;
    inl += in1;
  }
  // branch levels as the device runs them for root-only and incremental builds
  // (k_branch_fused: every encoding streamed block by block through a 17-word slot)
  for (int d = 63; d >= 0; --d) {
    for (uint64_t g = lbv[d]; g < lbv[d + 1]; ++g) {
      uint32_t j = lorder[g];
      uint32_t in1 = 0;
      uint64_t slot[LEAF_WORDS + 1];
      uint32_t p;
      if (lpos && (j & 1)) {  // a small level's path: records written, then read as a copy
        op_leaf_children(T, j);
        const uint64_t cb = T.br_cbase[j];
        p = op_branch_stream(T, j, slot, 1, &in1, ChildSrc{T.cmeta + cb, T.cref + 4 * cb, 1});
      } else {
        // (leaf positions: the child-table form, and every fourth branch the per-child form that
        // a wave with a branch spanning 4096+ keys takes on the device)
        p = T.kn ? op_branch_fused(T, j, slot, 1, &in1) : op_branch_stream(T, j, slot, 1, &in1, ChildSrc{}, (j & 3) == 0);
      }
      perms += p;
      hashes += branch_hash_count(T, j, p);
      inl += in1;
    }
  }
  memcpy(out_hash, res_hash.data(), nres * 32);
  memcpy(out_len, res_len.data(), nres * 4);
  memcpy(out_inl, res_inl.data(), nres * 32);
  if (stats_out) {
    stats_out[0] = m;
    stats_out[1] = B;
    stats_out[2] = hashes;
    stats_out[3] = perms;
    stats_out[4] = inl;
    stats_out[5] = ctr[CTR_EXT];
  }
  return 0;
}

extern "C" {

void emu_set_leaf_mode(int mode) { g_leaf_mode = mode; }
void emu_set_link_mode(int mode) { g_link_mode = mode; }
void emu_set_inject(int kind, uint64_t j) {
  g_inject = kind;
  g_inject_j = j;
}

int emu_build(const uint8_t* keys, const uint8_t* vals, const uint64_t* voff, uint64_t n, const uint32_t* seg,
              uint64_t nseg, uint32_t depth0, uint8_t* out_hash, uint32_t* out_len, uint8_t* out_inl,
              uint64_t* stats_out) {
  return build_core(keys, vals, voff, n, seg, nseg, depth0, out_hash, out_len, out_inl, stats_out);
}

int emu_node_children(const uint8_t* v, uint64_t len, int kind, uint8_t* out32, uint8_t* kinds, uint32_t* n) {
  uint8_t nc = 0;
  int st = op_node_children(v, (uint32_t)len, (uint8_t)kind, out32, kinds, &nc);
  *n = nc;
  return st;
}

void emu_kec256(const uint8_t* p, uint64_t len, uint8_t* out) {
  uint64_t h[4];
  kec256_msg<false>(p, (uint32_t)len, h);
  memcpy(out, h, 32);
}

void emu_synth(uint32_t cfg, uint64_t first, uint64_t n, uint8_t* addr, uint8_t* vals, uint64_t* voff) {
  uint64_t o = 0;
  for (uint64_t i = 0; i < n; ++i) {
    SynthAcct a = synth_acct(cfg, first + i);
    synth_addr_write(a, addr + 20 * i);
    voff[i] = o;
    o += synth_body_write(a, first + i, vals + o);
  }
  voff[n] = o;
}

int emu_fold16(const uint8_t* hash32x16, const uint32_t* len16, const uint8_t* inl32x16, uint8_t* out) {
  uint64_t refs[64];
  uint32_t lens[16];
  for (int i = 0; i < 16; ++i) {
    uint32_t L = len16[i];
    lens[i] = L == 0 ? 0 : (L >= 32 ? 32 : L);
    memcpy(refs + 4 * i, (L >= 32 ? hash32x16 : inl32x16) + 32 * i, 32);
  }
  uint64_t enc[80];
  uint32_t L = encode_branch16(refs, lens, (uint8_t*)enc);
  uint64_t h[4];
  kec256_msg<true>((const uint8_t*)enc, L, h);
  memcpy(out, h, 32);
  return 0;
}

}  // extern "C"

// The tile-local topology (topo_tiles: op_tile_ansv / op_tile_chain + the listed boundaries)
// against op_ansv + op_chain on every boundary, with small and full tiles, on the boundary
// values of sorted distinct keys (deep and shallow tries, segment breaks).  Returns 0 if
// pse (where the tiles keep it), psv / nsv of the representatives, rep, ord, isrep, glast and gk
// all agree.
extern "C" int emu_topo_tile_check(uint64_t seed, int iters) {
  std::mt19937_64 r(seed);
  const uint32_t tiles[] = {1, 7, 16, 64, 100, 1000, TOPO_TILE};
  for (int it = 0; it < iters; ++it) {
    const uint64_t n = 2 + r() % 20000;
    const int mode = it % 3;
    std::vector<std::array<uint8_t, 24>> keys(n);
    for (auto& k : keys)
      for (int d = 0; d < 24; ++d)  // mode 0: uniform nibbles; 1: narrow alphabets (deep); 2: mixed
        k[d] = (uint8_t)(mode == 0 ? r() % 16 : mode == 1 ? r() % (d < 8 ? 2 : 16) : r() % (1 + (d * 7 + r() % 3) % 16));
    std::sort(keys.begin(), keys.end());
    keys.erase(std::unique(keys.begin(), keys.end()), keys.end());
    const uint64_t nb = keys.size() - 1;
    if (nb == 0) continue;
    std::vector<uint8_t> u(nb + 16);
    for (uint64_t b = 0; b < nb; ++b) {
      int d = 0;
      while (d < 24 && keys[b][d] == keys[b + 1][d]) ++d;
      u[b] = (uint8_t)(d + 1);
      if (mode == 2 && r() % 500 == 0) u[b] = 0;  // a segment break
    }
    std::vector<std::vector<uint8_t>> lv;
    lv.reserve(8);
    Pyr P{};
    P.lv[0] = u.data();
    P.sz[0] = nb;
    P.nl = 1;
    while (P.sz[P.nl - 1] > 64) {
      uint64_t nin = P.sz[P.nl - 1], nout = (nin + 63) / 64;
      lv.emplace_back(nout + 16);
      for (uint64_t i = 0; i < nout; ++i) op_min64(P.lv[P.nl - 1], nin, lv.back().data(), i);
      P.lv[P.nl] = lv.back().data();
      P.sz[P.nl] = nout;
      P.nl++;
    }
    struct Arr {
      std::vector<int32_t> psv, nsv, pse;
      std::vector<uint32_t> rep, isrep;
      std::vector<uint8_t> ord, glast, gk;
      std::vector<unsigned long long> ctr;
      Topo T{};
      Arr(uint64_t nb, uint8_t* u)
          : psv(nb, 7), nsv(nb, 7), pse(nb, -7), rep(nb, 7), isrep(nb, 7), ord(nb, 7), glast(nb, 1), gk(nb, 0),
            ctr(CTR_N * CTR_SHARDS, 0) {
        T.u = u;
        T.psv = psv.data();
        T.nsv = nsv.data();
        T.pse = pse.data();
        T.rep = rep.data();
        T.isrep_bid = isrep.data();
        T.ord = ord.data();
        T.glast = glast.data();
        T.gk = gk.data();
        T.ctr = ctr.data();
      }
    };
    Arr G(nb, u.data()), L(nb, u.data());
    for (uint64_t b = 0; b < nb; ++b) op_ansv(G.T, P, b);
    for (uint64_t b = 0; b < nb; ++b) op_chain(G.T, b);
    topo_tiles(L.T, P, nb, tiles[it % 7]);
    if (G.ctr[CTR_ERR] || L.ctr[CTR_ERR]) return 1;
    for (uint64_t b = 0; b < nb; ++b) {
      if (u[b] == 0) continue;
      // (the tiles keep a link only where a walk from outside the tile can read it: -7 = not kept)
      if (L.pse[b] != -7 && G.pse[b] != L.pse[b]) return 2;
      if (G.rep[b] != L.rep[b] || G.ord[b] != L.ord[b] || G.isrep[b] != L.isrep[b]) return 3;
      if (G.glast[b] != L.glast[b]) return 4;
      if (G.rep[b] == b && (G.psv[b] != L.psv[b] || G.nsv[b] != L.nsv[b] || G.gk[b] != L.gk[b])) return 5;
    }
  }
  return 0;
}

// Brute-force check of the pyramid + SWAR nearest-smaller-value searches (trie_ops.h)
// against their naive definitions on random, shallow and almost-flat value arrays.
// Returns 0 if every query agrees.
#include <random>
extern "C" int emu_ansv_check(uint64_t seed, int iters) {
  std::mt19937_64 r(seed);
  for (int it = 0; it < iters; ++it) {
    uint64_t n = 1 + r() % 5000;
    std::vector<uint8_t> u(n + 16);
    int mode = it % 3;
    for (uint64_t i = 0; i < n; ++i)
      u[i] = mode == 0 ? r() % 65
                       : (mode == 1 ? 1 + (r() % 4 == 0 ? r() % 3 : 5 + r() % 3) : (r() % 100 == 0 ? 0 : 6 + r() % 2));
    std::vector<std::vector<uint8_t>> lv;
    lv.reserve(8);
    Pyr P{};
    P.lv[0] = u.data();
    P.sz[0] = n;
    P.nl = 1;
    while (P.sz[P.nl - 1] > 64) {
      uint64_t nin = P.sz[P.nl - 1], nout = (nin + 63) / 64;
      lv.emplace_back(nout + 16);
      for (uint64_t i = 0; i < nout; ++i) op_min64(P.lv[P.nl - 1], nin, lv.back().data(), i);
      P.lv[P.nl] = lv.back().data();
      P.sz[P.nl] = nout;
      P.nl++;
    }
    for (uint64_t b = 0; b < n; ++b) {
      uint32_t t = u[b];
      if (!t) continue;
      for (uint32_t tt : {t, t + 1}) {
        int64_t e = -1;
        for (int64_t j = (int64_t)b - 1; j >= 0; --j)
          if (u[j] < tt) {
            e = j;
            break;
          }
        if (ansv_left(P, b, tt) != e) return 1;
      }
      int64_t e = -1;
      for (uint64_t j = b + 1; j < n; ++j)
        if (u[j] < t) {
          e = (int64_t)j;
          break;
        }
      if (ansv_right(P, b, t) != e) return 2;
    }
  }
  return 0;
}

// The lane-spread permutation (keccak_xlane.h) replayed lane by lane -- each round's two
// steps over all 32 lanes of a group, with the LDS buffers as arrays -- against the
// one-thread permutation (keccak.h) on random states.  Returns the number of mismatches.
extern "C" int emu_xlane_check(uint64_t seed, int iters) {
  std::mt19937_64 r(seed);
  int bad = 0;
  XLane g[32];
  for (uint32_t l = 0; l < 32; ++l) g[l] = xlane_setup(l);
  for (int it = 0; it < iters; ++it) {
    KState S;
    uint64_t A[32] = {};
    for (int i = 0; i < 25; ++i) {
      A[i] = r();
      S.lo[i] = (uint32_t)A[i];
      S.hi[i] = (uint32_t)(A[i] >> 32);
    }
    for (uint32_t l = 25; l < 32; ++l) A[l] = r();  // lanes past the state carry garbage
    keccakf(S);
    for (int rd = 0; rd < 24; ++rd) {
      uint64_t bA[32], B[32];
      for (int l = 0; l < 32; ++l) bA[l] = A[l];
      for (int l = 0; l < 32; ++l) B[l] = xl_step_theta_rho(g[l], bA);
      for (int l = 0; l < 32; ++l) A[l] = xl_step_chi(g[l], B[l], B, rd);
    }
    for (int i = 0; i < 25; ++i) bad += A[i] != lane(S, i);
  }
  return bad;
}
