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
#include <cstring>
#include <numeric>
#include <string>
#include <vector>

#include "../../khipu_amd/csrc/nodedata.h"
#include "../../khipu_amd/csrc/resident.h"
#include "../../khipu_amd/csrc/synth.h"

using namespace khst;

// host mirror of IncArgs (khst.hip): the resident trie's tables
struct EmuTables {
  std::vector<uint64_t> ref, lref;
  std::vector<uint32_t> rlen, lrlen;
  std::vector<int8_t> lpd;
  std::vector<uint8_t> u;
  std::vector<std::vector<uint8_t>> pyr;
  std::vector<uint32_t> bid;
  uint64_t nb = 0;
  Pyr P() const {
    Pyr p{};
    if (nb == 0) return p;
    p.lv[0] = u.data();
    p.sz[0] = nb;
    p.nl = 1;
    for (auto& l : pyr) {
      p.lv[p.nl] = l.data();
      p.sz[p.nl] = l.size();
      p.nl++;
    }
    return p;
  }
};
struct EmuInc {
  const uint64_t* dkey = nullptr;  // nullptr: every branch dirty
  uint64_t nd = 0;
  Prev V{};
  EmuTables* out = nullptr;
};

// keys: n*32 (already keccak'd), vals/voff packed; seg nullable.
// Outputs per result r: hash (32 B), enc length, inline bytes (32 B).
// stats_out[0..5] = m, B, node hashes, node perms, inline nodes, extensions.
static int build_core(const uint8_t* keys, const uint8_t* vals, const uint64_t* voff, uint64_t n, const uint32_t* seg,
                      uint64_t nseg, uint32_t depth0, uint8_t* out_hash, uint32_t* out_len, uint8_t* out_inl,
                      uint64_t* stats_out, bool presorted, EmuInc* inc, std::vector<uint64_t>* skey_out,
                      std::vector<uint64_t>* svoff_out, std::vector<uint32_t>* svlen_out) {
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
  for (uint64_t i = 0; i < n; ++i) {
    bool dup_next = i + 1 < n && memcmp(keys + 32ull * order[i], keys + 32ull * order[i + 1], 32) == 0 &&
                    (!segmented || seg[order[i]] == seg[order[i + 1]]);
    if (!dup_next) sidx.push_back(order[i]);
  }
  if (presorted) {  // the merged set must already be sorted and unique (the device does not sort it)
    if (sidx.size() != n) return -1;
    for (uint64_t i = 0; i < n; ++i)
      if (sidx[i] != i) return -2;
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
  std::vector<uint8_t> u(nbb), ord(nbb), br_depth(nbb), br_ext(nbb), br_pord(nbb), lf_pord(m);
  std::vector<int32_t> psv(nbb), nsv(nbb), pse(nbb);
  std::vector<uint32_t> rep(nbb), isrep(nbb), br_k(nbb, 0), br_cbase(nbb), br_parent(nbb), br_first(nbb),
      br_len(nbb), ex_len(nbb), lf_parent(m), lf_len(m);
  std::vector<int8_t> lf_pd(m);
  std::vector<uint64_t> br_aoff(nbb), lf_aoff(m);
  std::vector<unsigned long long> ctr(CTR_N, 0);
  std::vector<uint32_t> hist(64, 0);
  T.u = u.data();
  T.psv = psv.data();
  T.nsv = nsv.data();
  T.pse = pse.data();
  T.rep = rep.data();
  T.ord = ord.data();
  T.isrep_bid = isrep.data();
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
  std::vector<std::vector<uint8_t>> pyr;
  Pyr P{};
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
    for (uint64_t b = 0; b < nb; ++b) op_ansv(T, P, b);
    for (uint64_t b = 0; b < nb; ++b) op_chain(T, b);
    if (ctr[CTR_ERR]) return -5;
    uint32_t run = 0;
    for (uint64_t b = 0; b < nb; ++b) {
      uint32_t f = isrep[b];
      isrep[b] = run;
      run += f;
    }
    B = run;
    for (uint64_t b = 0; b < nb; ++b) {
      op_branch_topo(T, P, nb, b);
      if (u[b] != 0 && rep[b] == b) {
        uint32_t j = isrep[b];
        hist[br_depth[j]]++;
        if (br_ext[j]) ctr[CTR_EXT]++;
      }
    }
  }
  // plain builds replay the device's early-leaf path (k_leaf_fused<true>: hashed from
  // the boundaries alone, references stashed, published after the topology)
  const bool early = inc == nullptr;
  std::vector<uint64_t> eref(early ? 4 * m + 4 : 0);
  std::vector<uint8_t> emeta(early ? m + 1 : 0);
  uint64_t perms = 0, hashes = 0, inl = 0, longb = 0;
  if (early) {
    T.lf_eref = eref.data();
    T.lf_emeta = emeta.data();
    for (uint64_t i = 0; i < m; ++i) {
      Key4 k = load_key(T.skey, i);
      const uint8_t* vp = T.vals + T.svoff[i];
      uint32_t vlen = T.svlen[i];
      int32_t pd = leaf_pd_early(T, i);
      LeafGeom g = leaf_geom(k, pd, vlen, vlen == 1 ? *vp : 0);
      if (g.L > LEAF_SHORT_MAX) {
        emeta[i] = EMETA_LONG;
        longb += (g.L + 7) & ~7u;
        continue;
      }
      uint64_t buf[LEAF_WORDS + 1] = {};
      BW w(buf, 1);
      leaf_header(w, k, g, vlen);
      w.bytes(vp, vlen);
      w.flush();
      uint32_t in1 = 0;
      uint32_t p = leaf_hash_early(T, i, pd == (int32_t)depth0 - 1, buf, 1, g.L, &in1);
      perms += p;
      hashes += p ? 1 : 0;
      inl += in1;
    }
  }
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
  for (uint64_t i = 0; i < m; ++i) {
    if (early)
      op_leaf_topo_early(T, i, bump);
    else
      op_leaf_topo(T, i, bump);
  }
  if (early && lfb != longb) return -7;  // the arena is sized by the early count
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
  if (inc) {
    inc->out->ref.assign(4 * B + 4, 0);
    inc->out->rlen.assign(B + 1, 0);
    T.br_ref = inc->out->ref.data();
    T.br_rlen = inc->out->rlen.data();
    inc->out->lref.assign(4 * m + 4, 0);
    inc->out->lrlen.assign(m + 1, 0);
    T.lf_ref = inc->out->lref.data();
    T.lf_rlen = inc->out->lrlen.data();
    if (inc->dkey) {
      T.lf_oldpos = inc->V.oldpos;
      T.lf_upd = inc->V.upd;
      T.lf_opd = inc->V.lpd;
      T.lf_oref = inc->V.lref;
      T.lf_orlen = inc->V.lrlen;
      T.br_dirty = br_dirty.data();
      for (uint64_t j = 0; j < B; ++j) op_br_dirty(T, inc->dkey, inc->nd, (uint32_t)j);
      for (uint64_t j = 0; j < B; ++j) op_br_clean(T, inc->V, (uint32_t)j);
      if (ctr[CTR_ERR]) return -6;
    }
  }
  T.arena = (uint8_t*)arena.data();
  if (!early)
    for (uint64_t i = 0; i < m; ++i) op_leaf_prep(T, i, T.vals + T.svoff[i], T.svlen[i]);
  for (uint64_t i = 0; i < m; ++i) {
    uint32_t in1 = 0;
    uint32_t p = early ? op_leaf_long(T, i, &in1) : op_leaf_hash(T, i, &in1);
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
      uint32_t p = op_branch_fused(T, j, slot, 1, &in1);
      perms += p;
      hashes += branch_hash_count(T, j, p);
      inl += in1;
    }
  }
  if (inc) {
    EmuTables& o = *inc->out;
    o.nb = nb;
    o.u.assign(u.begin(), u.begin() + nb);
    o.bid.assign(isrep.begin(), isrep.begin() + nb);
    o.pyr = pyr;
    o.lpd.assign(lf_pd.begin(), lf_pd.end());
  }
  if (skey_out) *skey_out = skey;
  if (svoff_out) *svoff_out = svoff;
  if (svlen_out) *svlen_out = svlen;
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

int emu_build(const uint8_t* keys, const uint8_t* vals, const uint64_t* voff, uint64_t n, const uint32_t* seg,
              uint64_t nseg, uint32_t depth0, uint8_t* out_hash, uint32_t* out_len, uint8_t* out_inl,
              uint64_t* stats_out) {
  return build_core(keys, vals, voff, n, seg, nseg, depth0, out_hash, out_len, out_inl, stats_out, false, nullptr,
                    nullptr, nullptr, nullptr);
}

// ---- resident trie replay (kh_trie_open / kh_trie_apply in khst.hip)
struct EmuTrie {
  std::vector<uint64_t> key, off;
  std::vector<uint8_t> val;
  uint64_t m = 0;
  EmuTables tab;
  uint8_t root[32];
};

static void emu_root_from(const uint8_t* h, uint32_t len, uint8_t* root) {
  static const uint8_t E[32] = {0x56, 0xe8, 0x1f, 0x17, 0x1b, 0xcc, 0x55, 0xa6, 0xff, 0x83, 0x45,
                                0xe6, 0x92, 0xc0, 0xf8, 0x6e, 0x5b, 0x48, 0xe0, 0x1b, 0x99, 0x6c,
                                0xad, 0xc0, 0x01, 0x62, 0x2f, 0xb5, 0xe3, 0x63, 0xb4, 0x21};
  memcpy(root, len ? h : E, 32);
}

void* emu_trie_open(const uint8_t* keys, const uint8_t* vals, const uint64_t* voff, uint64_t n, uint8_t* root) {
  EmuTrie* t = new EmuTrie();
  uint8_t hh[32], inl[32];
  uint32_t len = 0;
  EmuInc I;
  I.out = &t->tab;
  std::vector<uint64_t> svoff;
  std::vector<uint32_t> svlen;
  if (n) {
    if (build_core(keys, vals, voff, n, nullptr, 1, 0, hh, &len, inl, nullptr, false, &I, &t->key, &svoff, &svlen)) {
      delete t;
      return nullptr;
    }
  }
  t->m = t->key.size() / 4;
  t->off.assign(t->m + 1, 0);
  for (uint64_t i = 0; i < t->m; ++i) {
    t->off[i + 1] = t->off[i] + svlen[i];
    t->val.insert(t->val.end(), vals + svoff[i], vals + svoff[i] + svlen[i]);
  }
  emu_root_from(hh, len, t->root);
  memcpy(root, t->root, 32);
  return t;
}

// upsert keys: nup*32, values packed (up_off[nup+1]); delete keys: ndel*32.
// stats_out[0..3] = m', dirty keys, node hashes, node perms.
int emu_trie_apply(void* handle, const uint8_t* up_keys, const uint8_t* up_vals, const uint64_t* up_off, uint64_t nup,
                   const uint8_t* del_keys, uint64_t ndel, uint8_t* root, uint64_t* stats_out) {
  EmuTrie* t = (EmuTrie*)handle;
  const uint64_t nops = nup + ndel, m = t->m;
  std::vector<uint8_t> K(nops * 32 + 32);
  if (nup) memcpy(K.data(), up_keys, nup * 32);
  if (ndel) memcpy(K.data() + nup * 32, del_keys, ndel * 32);
  // sort + keep the last op per key (the device: sort_dedup)
  std::vector<uint32_t> order(nops);
  std::iota(order.begin(), order.end(), 0u);
  std::stable_sort(order.begin(), order.end(),
                   [&](uint32_t a, uint32_t b) { return memcmp(&K[32ull * a], &K[32ull * b], 32) < 0; });
  std::vector<uint32_t> oidx;
  for (uint64_t i = 0; i < nops; ++i)
    if (!(i + 1 < nops && memcmp(&K[32ull * order[i]], &K[32ull * order[i + 1]], 32) == 0)) oidx.push_back(order[i]);
  const uint64_t ns = oidx.size();
  std::vector<uint64_t> okey(4 * ns + 4);
  for (uint64_t o = 0; o < ns; ++o) memcpy(&okey[4 * o], &K[32ull * oidx[o]], 32);
  Merge M{};
  std::vector<uint32_t> o_lb(ns + 1), o_ins(ns + 1), o_eff(ns + 1), pos_cnt(m + 1, 0), pos_ins(m + 1),
      del_flag(m + 1, 0), pos_del(m + 1), pos_upd(m + 1, NONE);
  std::vector<uint8_t> o_kind(ns + 1);
  M.rkey = t->key.data();
  M.roff = t->off.data();
  M.m = m;
  M.okey = okey.data();
  M.oidx = oidx.data();
  M.nops = ns;
  M.nup = nup;
  M.uoff = up_off;
  M.o_lb = o_lb.data();
  M.o_kind = o_kind.data();
  M.o_ins = o_ins.data();
  M.o_eff = o_eff.data();
  M.pos_cnt = pos_cnt.data();
  M.pos_ins = pos_ins.data();
  M.pos_del = del_flag.data();
  M.pos_upd = pos_upd.data();
  for (uint64_t o = 0; o < ns; ++o) op_locate(M, o);
  for (uint64_t o = 0; o < ns; ++o) op_mark(M, o, [](uint32_t* p) { ++*p; });
  M.pos_del = pos_del.data();
  std::vector<uint32_t> o_insf(o_ins), o_efff(o_eff);
  auto excl = [](std::vector<uint32_t>& v, uint64_t n) {
    uint32_t r = 0;
    for (uint64_t i = 0; i < n; ++i) {
      uint32_t x = v[i];
      v[i] = r;
      r += x;
    }
    return r;
  };
  std::vector<uint32_t> tmp(pos_cnt);
  uint32_t n_ins = excl(tmp, m + 1);
  pos_ins = tmp;
  tmp = del_flag;
  uint32_t n_del = excl(tmp, m + 1);
  pos_del = tmp;
  M.pos_ins = pos_ins.data();
  M.pos_del = pos_del.data();
  excl(o_ins, ns);
  uint32_t nd = excl(o_eff, ns);
  const uint64_t m2 = m + n_ins - n_del;
  if (stats_out) {
    stats_out[0] = m2;
    stats_out[1] = nd;
    stats_out[2] = stats_out[3] = 0;
  }
  if (nd == 0) {
    memcpy(root, t->root, 32);
    return 0;
  }
  std::vector<uint64_t> nkey(4 * m2 + 4), nsrc(m2 + 1), dkey(4 * nd + 4);
  std::vector<uint32_t> nlen(m2 + 1), oldpos(m2 + 1);
  std::vector<uint8_t> nupd(m2 + 1);
  M.nkey = nkey.data();
  M.nlen = nlen.data();
  M.nsrc = nsrc.data();
  M.oldpos = oldpos.data();
  M.nupd = nupd.data();
  M.dkey = dkey.data();
  for (uint64_t j = 0; j < m; ++j) op_place_resident(M, del_flag.data(), j);
  for (uint64_t o = 0; o < ns; ++o) op_place_op(M, o_insf.data(), o_efff.data(), o);
  std::vector<uint64_t> noff(m2 + 1, 0);
  std::vector<uint8_t> nval;
  for (uint64_t i = 0; i < m2; ++i) {
    noff[i + 1] = noff[i] + nlen[i];
    uint64_t s = nsrc[i];
    const uint8_t* src = (s & SRC_UPSERT) ? up_vals + (s & ~SRC_UPSERT) : t->val.data() + s;
    nval.insert(nval.end(), src, src + nlen[i]);
  }
  nval.resize(nval.size() + 64);
  std::vector<uint8_t> nkb(32 * m2 + 32);
  memcpy(nkb.data(), nkey.data(), 32 * m2);
  EmuTables tab;
  EmuInc I;
  I.dkey = dkey.data();
  I.nd = nd;
  I.V.P = t->tab.P();
  I.V.bid = t->tab.bid.data();
  I.V.ref = t->tab.ref.data();
  I.V.rlen = t->tab.rlen.data();
  I.V.nb = t->tab.nb;
  I.V.oldpos = oldpos.data();
  I.V.upd = nupd.data();
  I.V.lpd = t->tab.lpd.data();
  I.V.lref = t->tab.lref.data();
  I.V.lrlen = t->tab.lrlen.data();
  I.out = &tab;
  uint8_t hh[32], inl[32];
  uint32_t len = 0;
  uint64_t st[6] = {0};
  if (m2) {
    int rc = build_core(nkb.data(), nval.data(), noff.data(), m2, nullptr, 1, 0, hh, &len, inl, st, true, &I, nullptr,
                        nullptr, nullptr);
    if (rc) return rc;
  }
  t->key.assign(nkey.begin(), nkey.begin() + 4 * m2);
  t->off = noff;
  t->val.assign(nval.begin(), nval.end() - 64);
  t->m = m2;
  t->tab = std::move(tab);
  emu_root_from(hh, len, t->root);
  memcpy(root, t->root, 32);
  if (stats_out) {
    stats_out[2] = st[2];
    stats_out[3] = st[3];
  }
  return 0;
}

void emu_trie_free(void* handle) { delete (EmuTrie*)handle; }

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
