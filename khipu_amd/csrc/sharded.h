// kh_trie_root_sharded: one state root over several GPUs of ONE process,
// for a caller that is not torch.distributed (the JVM through the C ABI).  Included at
// the end of khst.hip (it drives the same contexts, kernels and build).
//
// The trie is sharded by the top key nibble: shard g of N owns nibbles q with
// q * N >> 4 == g (2 per GPU at N = 8).  One call:
//   1. input slice g (contiguous, 1/N of the puts) is staged to device g, its keys
//      hashed there (KH_HASH_KEYS), and its records partitioned by owner
//      (kh_dev_partition: one stable 8-bit radix pass + a value copy);
//   2. exchange: every (source, owner) block of keys, value lengths and value bytes goes
//      over RCCL point-to-point (ncclSend / ncclRecv fused in groups: xGMI links, no host
//      staging), received source-major so "later put wins" holds.  The keys go first;
//      the lengths and value bytes follow on a stream of their own;
//   3. device g builds its nibbles' subtries from depth 1 (run_build, depth0 = 1) as soon
//      as its keys have landed: the key sort and the branch topology run while the
//      values are still in flight, the leaf stage waits for them (BuildArgs.vals_ready);
//   4. the 16 capped references are folded into the root branch on the host
//      (kh_fold_root16; MerklePatriciaTrie.scala:169: the root is always hashed).
// The reference-counts exchange and the 16-reference gather need no collective: one
// process holds every shard's host-side results.
//
// RCCL is loaded at run time (dlopen) so that libkhst.so loads without it; a process
// that already holds torch's RCCL reuses that copy.  A device list with REPEATED devices
// (several shards on one GPU: the topology the 1-GPU tests use to exercise the shard
// logic) moves the blocks with device-to-device copies instead, since one RCCL
// communicator cannot hold a device twice.
#pragma once
#include <dlfcn.h>
#include <rccl/rccl.h>

#include <chrono>
#include <exception>
#include <map>
#include <thread>

namespace khst {

struct Rccl {
  void* h = nullptr;
  ncclResult_t (*CommInitAll)(ncclComm_t*, int, const int*) = nullptr;
  ncclResult_t (*GroupStart)() = nullptr;
  ncclResult_t (*GroupEnd)() = nullptr;
  ncclResult_t (*Send)(const void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*Recv)(void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
  const char* (*ErrStr)(ncclResult_t) = nullptr;
};

static Rccl& rccl() {
  static Rccl R;
  static std::once_flag once;
  std::call_once(once, [] {
    void* h = dlopen("librccl.so", RTLD_NOW | RTLD_NOLOAD);  // torch's copy, if loaded
    if (!h) h = dlopen("librccl.so.1", RTLD_NOW);
    if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW);
    if (!h) return;
    R.CommInitAll = (decltype(R.CommInitAll))dlsym(h, "ncclCommInitAll");
    R.GroupStart = (decltype(R.GroupStart))dlsym(h, "ncclGroupStart");
    R.GroupEnd = (decltype(R.GroupEnd))dlsym(h, "ncclGroupEnd");
    R.Send = (decltype(R.Send))dlsym(h, "ncclSend");
    R.Recv = (decltype(R.Recv))dlsym(h, "ncclRecv");
    R.ErrStr = (decltype(R.ErrStr))dlsym(h, "ncclGetErrorString");
    if (R.CommInitAll && R.GroupStart && R.GroupEnd && R.Send && R.Recv && R.ErrStr) R.h = h;
  });
  if (!R.h) throw KhError{KH_EDEVICE, "RCCL (librccl.so) not found: the sharded root needs it"};
  return R;
}
#define NCCLCHK(x)                                                                              \
  do {                                                                                          \
    ncclResult_t r_ = (x);                                                                      \
    if (r_ != ncclSuccess) throw KhError{KH_EDEVICE, std::string("RCCL: ") + rccl().ErrStr(r_)}; \
  } while (0)

// per-shard state, kept between calls (HBM buffers grow, never shrink)
struct Shard {
  kh_ctx* c = nullptr;  // private context (shards may share a device)
  DevBuf k32, pk, pv, pl, rk, rv, rl, rvo, vscan;
  hipStream_t cs = nullptr;      // value exchange + offsets (beside the build's streams)
  hipEvent_t ev_vals = nullptr;  // ... done
  ~Shard() {
    if (cs) (void)hipStreamDestroy(cs);
    if (ev_vals) (void)hipEventDestroy(ev_vals);
    if (c) kh_ctx_destroy(c);
  }
  uint64_t lo = 0, n = 0;            // input slice
  uint64_t cnt[16] = {}, nb[16] = {};  // records / value bytes for each owner
  uint64_t m = 0, mb = 0;            // received records / value bytes
  BuildOut O;
  kh_stats st{};
};
static std::mutex g_shard_mu;  // one sharded call at a time (shards and communicators are shared)
static std::vector<Shard*> g_shards;
static std::map<std::vector<int>, std::vector<ncclComm_t>> g_comms;

static uint32_t owner_of_nibble(uint32_t q, uint32_t N) { return (q * N) >> 4; }

template <typename Fn>
static void on_shards(std::vector<Shard*>& S, const std::vector<int>& dev, Fn fn) {
  std::vector<std::exception_ptr> err(S.size());
  std::vector<std::thread> th;
  for (size_t g = 0; g < S.size(); ++g)
    th.emplace_back([&, g] {
      try {
        HIPCHK(hipSetDevice(dev[g]));
        fn(g, *S[g]);
      } catch (...) {
        err[g] = std::current_exception();
      }
    });
  for (auto& t : th) t.join();
  for (auto& e : err)
    if (e) std::rethrow_exception(e);
}

static void sharded_root(const int* devices, int ngpus, const uint8_t* keys, uint32_t klen, const uint8_t* vals,
                         const uint64_t* voff, uint64_t n, uint32_t flags, uint8_t* root32, kh_stats* stats) {
  if (ngpus < 1 || ngpus > 16) throw KhError{KH_EINVAL, "ngpus must be in [1, 16]"};
  if (!(flags & KH_HASH_KEYS) && klen != 32) throw KhError{KH_EINVAL, "keys must be 32 bytes unless KH_HASH_KEYS"};
  const uint32_t N = (uint32_t)ngpus;
  std::vector<int> dev(devices, devices + N);
  int ndev = 0;
  HIPCHK(hipGetDeviceCount(&ndev));
  bool distinct = true;
  for (uint32_t g = 0; g < N; ++g) {
    if (dev[g] < 0 || dev[g] >= ndev) throw KhError{KH_EDEVICE, "no such device"};
    for (uint32_t h = 0; h < g; ++h) distinct &= dev[h] != dev[g];
  }
  std::lock_guard<std::mutex> lk(g_shard_mu);
  const auto t0 = std::chrono::steady_clock::now();
  auto ms_since = [](std::chrono::steady_clock::time_point a) {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - a).count();
  };
  while (g_shards.size() < N) g_shards.push_back(new Shard());
  std::vector<Shard*> S(g_shards.begin(), g_shards.begin() + N);
  for (uint32_t g = 0; g < N; ++g) {
    if (S[g]->c && S[g]->c->dev != dev[g]) {  // re-home the slot on its new device
      delete S[g];
      S[g] = g_shards[g] = new Shard();
    }
    if (!S[g]->c) {
      S[g]->c = ctx_new(dev[g]);
      HIPCHK(hipSetDevice(dev[g]));
      HIPCHK(hipStreamCreateWithFlags(&S[g]->cs, hipStreamNonBlocking));
      HIPCHK(hipEventCreateWithFlags(&S[g]->ev_vals, hipEventDisableTiming));
    }
    S[g]->lo = n * g / N;
    S[g]->n = n * (g + 1) / N - S[g]->lo;
  }
  // KH_SHARD_RCCL: the RCCL exchange even for a list that repeats a device (a communicator that
  // accepts repeats: the tests' in-process loopback, tests/loopback) -- the JVM's distinct-device
  // path run on a one-GPU box
  const bool use_rccl = distinct || (flags & KH_SHARD_RCCL);
  std::vector<ncclComm_t>* comms = nullptr;
  if (use_rccl) {
    Rccl& R = rccl();
    auto it = g_comms.find(dev);
    if (it == g_comms.end()) {
      std::vector<ncclComm_t> cm(N);
      NCCLCHK(R.CommInitAll(cm.data(), (int)N, dev.data()));
      it = g_comms.emplace(dev, cm).first;
    }
    comms = &it->second;
  }

  // ---- 1. stage, hash, partition (every shard in parallel)
  on_shards(S, dev, [&](size_t, Shard& s) {
    kh_ctx* c = s.c;
    memset(s.cnt, 0, sizeof(s.cnt));
    memset(s.nb, 0, sizeof(s.nb));
    if (!s.n) return;
    Staged in = stage_inputs(c, keys + s.lo * klen, klen, vals, voff + s.lo, s.n, nullptr);
    const uint8_t* K = in.keys;
    if (flags & KH_HASH_KEYS) {
      s.k32.ensure(s.n * 32 + 64, c->dev);
      if (klen <= 135)
        hipLaunchKernelGGL(k_hash_keys<true>, GRID(s.n, BS), dim3(BS), 0, c->st, in.keys, klen, s.n, (uint64_t*)s.k32.p);
      else
        hipLaunchKernelGGL(k_hash_keys<false>, GRID(s.n, BS), dim3(BS), 0, c->st, in.keys, klen, s.n, (uint64_t*)s.k32.p);
      LAUNCH_CHECK();
      K = (const uint8_t*)s.k32.p;
    }
    const uint64_t vb = voff[s.lo + s.n] - voff[s.lo];
    s.pk.ensure(s.n * 32 + 64, c->dev);
    s.pv.ensure(vb + 64, c->dev);
    s.pl.ensure(s.n * 8 + 64, c->dev);
    int rc = kh_dev_partition(c, K, in.vals, in.voff, s.n, N, (uint8_t*)s.pk.p, (uint8_t*)s.pv.p, (uint64_t*)s.pl.p,
                              s.cnt, s.nb);
    if (rc != KH_OK) throw KhError{rc, "partition: " + g_err};
  });
  const double t_part = ms_since(t0);

  // ---- 2. exchange: owner p receives every source g's block, source-major
  std::vector<uint64_t> roff((size_t)N * N), rboff((size_t)N * N), soff((size_t)N * N), sboff((size_t)N * N);
  for (uint32_t p = 0; p < N; ++p) {
    uint64_t m = 0, mb = 0;
    for (uint32_t g = 0; g < N; ++g) {
      roff[p * N + g] = m;
      rboff[p * N + g] = mb;
      m += S[g]->cnt[p];
      mb += S[g]->nb[p];
    }
    S[p]->m = m;
    S[p]->mb = mb;
    // receive buffers live on the OWNER's device (this loop runs on the caller's thread)
    const int pd = S[p]->c->dev;
    S[p]->rk.ensure(m * 32 + 64, pd);
    S[p]->rl.ensure(m * 8 + 64, pd);
    S[p]->rv.ensure(mb + 64, pd);
    S[p]->rvo.ensure((m + 1) * 8 + 64, pd);
  }
  for (uint32_t g = 0; g < N; ++g) {
    uint64_t o = 0, ob = 0;
    for (uint32_t p = 0; p < N; ++p) {
      soff[g * N + p] = o;
      sboff[g * N + p] = ob;
      o += S[g]->cnt[p];
      ob += S[g]->nb[p];
    }
  }
  const auto t1 = std::chrono::steady_clock::now();
  for (uint32_t p = 0; p < N; ++p) S[p]->vscan.ensure(scan_scratch_bytes(S[p]->m, 8) + 256, S[p]->c->dev);
  // the offsets of the received values, on the shard's exchange stream once its lengths
  // and bytes have landed; the build's leaf stage waits for ev_vals
  auto value_offsets = [&](Shard& s) {
    HIPCHK(hipSetDevice(s.c->dev));
    if (s.m)
      scan_exclusive<uint64_t>((const uint64_t*)s.rl.p, (uint64_t*)s.rvo.p, s.m, (uint64_t*)s.rvo.p + s.m, s.vscan.p,
                               s.cs);
    HIPCHK(hipEventRecord(s.ev_vals, s.cs));
  };
  if (use_rccl) {
    Rccl& R = rccl();
    for (int part = 0; part < 2; ++part) {  // 0: keys (build streams), 1: lengths + values (exchange streams)
      NCCLCHK(R.GroupStart());
      for (uint32_t g = 0; g < N; ++g)
        for (uint32_t p = 0; p < N; ++p) {
          const uint64_t c = S[g]->cnt[p], b = S[g]->nb[p];
          if (!c) continue;  // both sides know the block sizes
          Shard& src = *S[g];
          Shard& dst = *S[p];
          ncclComm_t cs = (*comms)[g], cd = (*comms)[p];
          if (part == 0) {
            NCCLCHK(R.Send((uint8_t*)src.pk.p + soff[g * N + p] * 32, c * 32, ncclUint8, (int)p, cs, src.c->st));
            NCCLCHK(R.Recv((uint8_t*)dst.rk.p + roff[p * N + g] * 32, c * 32, ncclUint8, (int)g, cd, dst.c->st));
            continue;
          }
          NCCLCHK(R.Send((uint64_t*)src.pl.p + soff[g * N + p], c, ncclUint64, (int)p, cs, src.cs));
          NCCLCHK(R.Recv((uint64_t*)dst.rl.p + roff[p * N + g], c, ncclUint64, (int)g, cd, dst.cs));
          if (b) {
            NCCLCHK(R.Send((uint8_t*)src.pv.p + sboff[g * N + p], b, ncclUint8, (int)p, cs, src.cs));
            NCCLCHK(R.Recv((uint8_t*)dst.rv.p + rboff[p * N + g], b, ncclUint8, (int)g, cd, dst.cs));
          }
        }
      NCCLCHK(R.GroupEnd());
    }
    for (uint32_t g = 0; g < N; ++g) value_offsets(*S[g]);
  } else {
    // shards sharing devices: same-device or peer copies, ordered on the sources' streams,
    // every block landed before any build starts
    for (uint32_t g = 0; g < N; ++g) {
      Shard& src = *S[g];
      HIPCHK(hipSetDevice(dev[g]));
      for (uint32_t p = 0; p < N; ++p) {
        const uint64_t c = src.cnt[p], b = src.nb[p];
        if (!c) continue;
        Shard& dst = *S[p];
        HIPCHK(hipMemcpyPeerAsync((uint8_t*)dst.rk.p + roff[p * N + g] * 32, dev[p],
                                  (uint8_t*)src.pk.p + soff[g * N + p] * 32, dev[g], c * 32, src.c->st));
        HIPCHK(hipMemcpyPeerAsync((uint64_t*)dst.rl.p + roff[p * N + g], dev[p], (uint64_t*)src.pl.p + soff[g * N + p],
                                  dev[g], c * 8, src.c->st));
        if (b)
          HIPCHK(hipMemcpyPeerAsync((uint8_t*)dst.rv.p + rboff[p * N + g], dev[p],
                                    (uint8_t*)src.pv.p + sboff[g * N + p], dev[g], b, src.c->st));
      }
    }
    for (uint32_t g = 0; g < N; ++g) {
      HIPCHK(hipSetDevice(dev[g]));
      HIPCHK(hipStreamSynchronize(S[g]->c->st));
    }
    for (uint32_t g = 0; g < N; ++g) value_offsets(*S[g]);
  }
  for (uint32_t g = 0; g < N; ++g) {  // the keys have landed (the values may still be in flight)
    HIPCHK(hipSetDevice(dev[g]));
    HIPCHK(hipStreamSynchronize(S[g]->c->st));
  }
  const double t_xchg = ms_since(t1);

  // ---- 3. the owned subtries from nibble 1 (every shard in parallel)
  const auto t2 = std::chrono::steady_clock::now();
  on_shards(S, dev, [&](size_t, Shard& s) {
    kh_ctx* c = s.c;
    s.O = BuildOut{};
    memset(&s.st, 0, sizeof(s.st));
    if (!s.m) {
      s.O.res_hash.assign(16 * 4, 0);
      s.O.res_len.assign(16, 0);
      s.O.res_inl.assign(16 * 4, 0);
      return;
    }
    BuildArgs A{(const uint8_t*)s.rk.p, 32, (const uint8_t*)s.rv.p, (const uint64_t*)s.rvo.p, s.m, nullptr, 1, 1, 0,
                false};
    A.vals_ready = s.ev_vals;
    run_build(c, A, s.O, &s.st);
  });
  const double t_build = ms_since(t2);

  // ---- 4. fold the 16 references (each from its nibble's owner)
  uint8_t H[16 * 32], I[16 * 32];
  uint32_t L[16];
  int occupied = 0, last = -1;
  for (uint32_t q = 0; q < 16; ++q) {
    const Shard& o = *S[owner_of_nibble(q, N)];
    memcpy(H + 32 * q, &o.O.res_hash[4 * q], 32);
    memcpy(I + 32 * q, &o.O.res_inl[4 * q], 32);
    L[q] = o.O.res_len[q];
    if (L[q]) ++occupied, last = (int)q;
  }
  uint64_t extra_hashes = 0;
  if (occupied >= 2) {
    int rc = kh_fold_root16(H, L, I, root32);
    if (rc != KH_OK) throw KhError{rc, g_err};
    extra_hashes = 1;
  } else if (occupied == 0) {
    memcpy(root32, EMPTY_TRIE_HASH, 32);
  } else {  // the root is not a branch: the one occupied nibble's owner holds every key
    Shard& s = *S[owner_of_nibble((uint32_t)last, N)];
    HIPCHK(hipSetDevice(s.c->dev));
    BuildArgs A{(const uint8_t*)s.rk.p, 32, (const uint8_t*)s.rv.p, (const uint64_t*)s.rvo.p, s.m, nullptr, 1, 0, 0,
                false};
    BuildOut O;
    run_build(s.c, A, O, &s.st);
    copy_root(O, 0, root32);
  }
  if (stats) {
    memset(stats, 0, sizeof(*stats));
    stats->n_inputs = n;
    for (uint32_t g = 0; g < N; ++g) {
      const kh_stats& t = S[g]->st;
      stats->n_leaves += t.n_leaves;
      stats->n_branches += t.n_branches;
      stats->n_extensions += t.n_extensions;
      stats->n_inline += t.n_inline;
      stats->n_node_hashes += t.n_node_hashes;
      stats->n_node_perms += t.n_node_perms;
      stats->arena_bytes += t.arena_bytes;
      stats->n_levels = std::max(stats->n_levels, t.n_levels);
      stats->full_sort |= t.full_sort;
      stats->t_leaf_ms = std::max(stats->t_leaf_ms, t.t_leaf_ms);
      stats->t_branch_ms = std::max(stats->t_branch_ms, t.t_branch_ms);
      stats->t_topo_ms = std::max(stats->t_topo_ms, t.t_topo_ms);
    }
    stats->n_branches += extra_hashes;
    stats->n_node_hashes += extra_hashes;
    stats->n_key_perms = (flags & KH_HASH_KEYS) ? n * (uint64_t)(klen / 136 + 1) : 0;
    // host wall clock of the phases (the shards run concurrently)
    stats->t_keys_ms = t_part;   // stage + key hashing + partition
    stats->t_sort_ms = t_xchg;   // the key exchange (the values land during the build)
    stats->t_total_ms = ms_since(t0);
    (void)t_build;
  }
}

// Many independent tries (configs[3]: every contract's storage trie, TrieStorage.flush per
// contract via BlockWorldState.scala:243-252) over several GPUs of one process (SURVEY §8e
// "Other configs"): the tries are split into ngpus contiguous ranges of about equal slot
// counts; each device stages and builds its range as one segmented build; the roots land in
// roots32 in trie order.  No exchange: the tries are independent.
static void segmented_sharded(const int* devices, int ngpus, const uint8_t* keys, uint32_t klen, const uint8_t* vals,
                              const uint64_t* voff, const uint64_t* seg_off, uint64_t nseg, uint32_t flags,
                              uint8_t* roots32, kh_stats* stats) {
  if (ngpus < 1 || ngpus > 16) throw KhError{KH_EINVAL, "ngpus must be in [1, 16]"};
  const uint32_t N = (uint32_t)ngpus;
  std::vector<int> dev(devices, devices + N);
  int ndev = 0;
  HIPCHK(hipGetDeviceCount(&ndev));
  for (uint32_t g = 0; g < N; ++g)
    if (dev[g] < 0 || dev[g] >= ndev) throw KhError{KH_EDEVICE, "no such device"};
  for (uint64_t s = 0; s < nseg; ++s)
    if (seg_off[s + 1] < seg_off[s]) throw KhError{KH_EINVAL, "seg_off not monotone"};
  // trie ranges [b[g], b[g+1]) balanced by slots
  const uint64_t tot = seg_off[nseg] - seg_off[0];
  std::vector<uint64_t> b(N + 1, nseg);
  b[0] = 0;
  for (uint32_t g = 1; g < N; ++g) {
    const uint64_t want = seg_off[0] + tot * g / N;
    b[g] = (uint64_t)(std::lower_bound(seg_off, seg_off + nseg, want) - seg_off);
    if (b[g] < b[g - 1]) b[g] = b[g - 1];
  }
  std::lock_guard<std::mutex> lk(g_shard_mu);
  while (g_shards.size() < N) g_shards.push_back(new Shard());
  std::vector<Shard*> S(g_shards.begin(), g_shards.begin() + N);
  for (uint32_t g = 0; g < N; ++g) {
    if (S[g]->c && S[g]->c->dev != dev[g]) {
      delete S[g];
      S[g] = g_shards[g] = new Shard();
    }
    if (!S[g]->c) {
      S[g]->c = ctx_new(dev[g]);
      HIPCHK(hipSetDevice(dev[g]));
      HIPCHK(hipStreamCreateWithFlags(&S[g]->cs, hipStreamNonBlocking));
      HIPCHK(hipEventCreateWithFlags(&S[g]->ev_vals, hipEventDisableTiming));
    }
  }
  const auto t0 = std::chrono::steady_clock::now();
  on_shards(S, dev, [&](size_t g, Shard& s) {
    memset(&s.st, 0, sizeof(s.st));
    const uint64_t lo = b[g], hi = b[g + 1], ns = hi - lo;
    if (ns == 0) return;
    const uint64_t i0 = seg_off[lo], n = seg_off[hi] - i0;
    if (n == 0) {
      for (uint64_t t = lo; t < hi; ++t) memcpy(roots32 + 32 * t, EMPTY_TRIE_HASH, 32);
      return;
    }
    std::vector<uint32_t> seg(n);
    for (uint64_t t = lo; t < hi; ++t)
      for (uint64_t i = seg_off[t]; i < seg_off[t + 1]; ++i) seg[i - i0] = (uint32_t)(t - lo);
    Staged in = stage_inputs(s.c, keys + i0 * klen, klen, vals, voff + i0, n, &seg);
    BuildArgs A{in.keys, klen, in.vals, in.voff, n, in.seg, ns, 0, flags, false};
    BuildOut O;
    run_build(s.c, A, O, &s.st);
    for (uint64_t t = lo; t < hi; ++t) copy_root(O, t - lo, roots32 + 32 * t);
  });
  if (stats) {
    memset(stats, 0, sizeof(*stats));
    stats->n_inputs = tot;
    for (uint32_t g = 0; g < N; ++g) {
      const kh_stats& t = S[g]->st;
      stats->n_leaves += t.n_leaves;
      stats->n_branches += t.n_branches;
      stats->n_extensions += t.n_extensions;
      stats->n_inline += t.n_inline;
      stats->n_node_hashes += t.n_node_hashes;
      stats->n_node_perms += t.n_node_perms;
      stats->n_key_perms += t.n_key_perms;
      stats->n_levels = std::max(stats->n_levels, t.n_levels);
      stats->t_leaf_ms = std::max(stats->t_leaf_ms, t.t_leaf_ms);
      stats->t_branch_ms = std::max(stats->t_branch_ms, t.t_branch_ms);
      stats->t_topo_ms = std::max(stats->t_topo_ms, t.t_topo_ms);
      stats->t_sort_ms = std::max(stats->t_sort_ms, t.t_sort_ms);
      stats->t_keys_ms = std::max(stats->t_keys_ms, t.t_keys_ms);
    }
    stats->t_total_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  }
}

}  // namespace khst

extern "C" int kh_trie_roots_segmented_sharded(const int* devices, int ngpus, const uint8_t* keys, uint32_t klen,
                                               const uint8_t* vals, const uint64_t* voff, const uint64_t* seg_off,
                                               uint64_t nseg, uint32_t flags, uint8_t* roots32, kh_stats* stats) {
  API_TRY({
    if (!devices) throw KhError{KH_EINVAL, "null device list"};
    if (nseg == 0) return KH_OK;
    if (!seg_off || !roots32 || (seg_off[nseg] > seg_off[0] && (!keys || !voff)))
      throw KhError{KH_EINVAL, "null input"};
    khst::segmented_sharded(devices, ngpus, keys, klen, vals, voff, seg_off, nseg, flags, roots32, stats);
  })
}

extern "C" int kh_trie_root_sharded(const int* devices, int ngpus, const uint8_t* keys, uint32_t klen,
                                    const uint8_t* vals, const uint64_t* voff, uint64_t n, uint32_t flags,
                                    uint8_t root32[32], kh_stats* stats) {
  API_TRY({
    if (n && (!keys || !voff)) throw KhError{KH_EINVAL, "null input"};
    if (!devices) throw KhError{KH_EINVAL, "null device list"};
    khst::sharded_root(devices, ngpus, keys, klen, vals, voff, n, flags, root32, stats);
  })
}
