// Device primitives for the state-root pipeline: wave reductions, exclusive scan,
// and a stable LSD radix sort of (uint64 key, uint32 value) pairs.
//
// Radix sort: 8-bit digits; one launch counts the digits of every pass, then one launch per
// pass (decoupled look-back over the tiles' digit counts).  A tile is 256 threads x 16 keys
// (4 for small sorts); each 64-lane wave owns a contiguous slice of the tile and ranks its
// keys with a ballot-based wave-level multisplit (8 ballots give the mask of lanes holding
// the same digit), so the scatter is stable; the tile is then staged in LDS in digit order
// and written out run by run (coalesced).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "wave.h"

namespace khst {

// ---------------------------------------------------------------------------
// Exclusive scan (T = uint32_t or uint64_t).  256 threads x 8 items per tile.
// ---------------------------------------------------------------------------
constexpr int SCAN_THREADS = 256;
constexpr int SCAN_ITEMS = 8;
constexpr int SCAN_TILE = SCAN_THREADS * SCAN_ITEMS;

template <typename T>
__device__ __forceinline__ T block_exclusive_scan(T v, T* lds_waves, T* total) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  T x = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    T y = __shfl_up(x, o);
    if (lane >= o) x += y;
  }
  if (lane == 63) lds_waves[w] = x;
  __syncthreads();
  T wbase = 0, tot = 0;
#pragma unroll
  for (int i = 0; i < SCAN_THREADS / 64; ++i) {
    T s = lds_waves[i];
    if (i < w) wbase += s;
    tot += s;
  }
  __syncthreads();
  *total = tot;
  return wbase + x - v;
}

// n_dev (nullable): a device count that caps n (the entries past it are neither read nor
// written; their tiles' sums are 0)
__device__ __forceinline__ uint64_t scan_n(uint64_t n, const uint32_t* n_dev) {
  return n_dev && (uint64_t)*n_dev < n ? (uint64_t)*n_dev : n;
}

template <typename T>
__global__ void __launch_bounds__(SCAN_THREADS) k_scan_tiles(const T* in, T* out, uint64_t n, T* tile_sums,
                                                             T* last_in, const uint32_t* n_dev) {
  topo_prio();
  n = scan_n(n, n_dev);
  __shared__ T lw[SCAN_THREADS / 64];
  uint64_t base = (uint64_t)blockIdx.x * SCAN_TILE + (uint64_t)threadIdx.x * SCAN_ITEMS;
  T v[SCAN_ITEMS];
  T s = 0;
#pragma unroll
  for (int i = 0; i < SCAN_ITEMS; ++i) {
    v[i] = (base + i < n) ? in[base + i] : (T)0;
    if (last_in && base + i == n - 1) *last_in = v[i];  // read before any output of this tile lands
    s += v[i];
  }
  T tot;
  T ex = block_exclusive_scan<T>(s, lw, &tot);
#pragma unroll
  for (int i = 0; i < SCAN_ITEMS; ++i) {
    if (base + i < n) out[base + i] = ex;
    ex += v[i];
  }
  if (threadIdx.x == 0) tile_sums[blockIdx.x] = tot;
}

template <typename T>
__global__ void __launch_bounds__(SCAN_THREADS) k_scan_add(T* out, uint64_t n, const T* tile_off,
                                                           const uint32_t* n_dev) {
  topo_prio();
  n = scan_n(n, n_dev);
  uint64_t base = (uint64_t)blockIdx.x * SCAN_TILE;
  if (base >= n) return;
  T add = tile_off[blockIdx.x];
  for (int i = threadIdx.x; i < SCAN_TILE; i += SCAN_THREADS)
    if (base + i < n) out[base + i] += add;
}

template <typename T>
__global__ void k_scan_total(const T* in_last, const T* out, uint64_t n, T* total, const uint32_t* n_dev) {
  topo_prio();
  n = scan_n(n, n_dev);
  *total = n ? *in_last + out[n - 1] : (T)0;
}

// Small scans (a block commit's op and element counts): one block walks the tiles in order
// carrying the running sum, one launch instead of the tile / recursive / add / total chain
// (each launch of that chain costs ~5 us of dispatch at these sizes).  A tile is loaded
// coalesced (element i * 1024 + thread) and transposed through LDS so that each thread
// scans SMALL_ITEMS consecutive elements; the next tile's loads are in flight during the
// current tile's scan.  (Loaded thread-contiguous instead, one CU's vector memory path ran
// at ~13 us per 8192-element tile: profiles/r3w_block_commit_trace_50m.json.)
constexpr int SCAN_SMALL_THREADS = 1024;
constexpr uint64_t SCAN_SMALL_MAX = 32768;
template <typename T>
__device__ __forceinline__ void scan_small_block(const T* in, T* out, uint64_t n, T* total) {
  constexpr int IT = sizeof(T) == 8 ? 4 : 8;  // items per thread (LDS: 32 KiB + padding)
  constexpr uint32_t TILE = SCAN_SMALL_THREADS * IT;
  __shared__ T buf[TILE + TILE / 32];  // element p at p + p / 32 (the thread-contiguous reads
                                       // then fall in distinct banks)
  __shared__ T lw[SCAN_SMALL_THREADS / 64];
  const uint32_t tid = threadIdx.x;
  const int lane = tid & 63, w = tid >> 6;
  T carry = 0;
  T v[IT];
  auto load = [&](uint64_t t0) {
#pragma unroll
    for (int i = 0; i < IT; ++i) {
      const uint64_t idx = t0 + (uint64_t)i * SCAN_SMALL_THREADS + tid;
      v[i] = idx < n ? in[idx] : (T)0;
    }
  };
  auto at = [](uint32_t p) { return p + (p >> 5); };
  load(0);
  for (uint64_t t0 = 0; t0 < n; t0 += TILE) {
#pragma unroll
    for (int i = 0; i < IT; ++i) buf[at(i * SCAN_SMALL_THREADS + tid)] = v[i];
    __syncthreads();
    if (t0 + TILE < n) load(t0 + TILE);  // (in == out: a later tile's inputs)
    T cur[IT];
    T s = 0;
#pragma unroll
    for (int j = 0; j < IT; ++j) {
      cur[j] = buf[at(tid * IT + j)];
      s += cur[j];
    }
    T x = s;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      T y = __shfl_up(x, o);
      if (lane >= o) x += y;
    }
    if (lane == 63) lw[w] = x;
    __syncthreads();
    T wbase = 0, tot = 0;
#pragma unroll
    for (int i = 0; i < SCAN_SMALL_THREADS / 64; ++i) {
      const T q = lw[i];
      if (i < w) wbase += q;
      tot += q;
    }
    T ex = carry + wbase + x - s;
#pragma unroll
    for (int j = 0; j < IT; ++j) {
      buf[at(tid * IT + j)] = ex;
      ex += cur[j];
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < IT; ++i) {
      const uint32_t p = i * SCAN_SMALL_THREADS + tid;
      if (t0 + p < n) out[t0 + p] = buf[at(p)];
    }
    carry += tot;
    __syncthreads();  // buf and lw are rewritten by the next tile
  }
  if (total && tid == 0) *total = carry;
}
template <typename T>
__global__ void __launch_bounds__(SCAN_SMALL_THREADS) k_scan_small(const T* in, T* out, uint64_t n, T* total) {
  topo_prio();
  scan_small_block<T>(in, out, n, total);
}
// Up to three small scans of n elements in one launch, one block each (a commit's per-op
// flags: new-trie starts, upsert ranks, value offsets); a null input skips its block.
struct ScanJob {
  const void* in;
  void* out;
  void* total;
  bool wide;  // uint64_t elements (else uint32_t)
};
__global__ void __launch_bounds__(SCAN_SMALL_THREADS) k_scan_small3(ScanJob a, ScanJob b, ScanJob c, uint64_t n) {
  topo_prio();
  const ScanJob& j = blockIdx.x == 0 ? a : blockIdx.x == 1 ? b : c;
  if (!j.in) return;
  if (j.wide)
    scan_small_block<uint64_t>((const uint64_t*)j.in, (uint64_t*)j.out, n, (uint64_t*)j.total);
  else
    scan_small_block<uint32_t>((const uint32_t*)j.in, (uint32_t*)j.out, n, (uint32_t*)j.total);
}

// Mid-size scans (up to SCAN_TWO_MAX_TILES tiles): after k_scan_tiles, each block sums the
// tile sums before it itself (no recursive scan of the sums) and adds them; the last block
// writes the total.  Two launches.
constexpr uint64_t SCAN_TWO_MAX_TILES = 2048;
template <typename T>
__global__ void __launch_bounds__(SCAN_THREADS) k_scan_add_sums(T* out, uint64_t n, const T* sums, uint32_t tiles,
                                                                T* total, const uint32_t* n_dev) {
  topo_prio();
  n = scan_n(n, n_dev);
  __shared__ T lw[SCAN_THREADS / 64];
  const uint32_t b = blockIdx.x;
  T s = 0;
  for (uint32_t t = threadIdx.x; t < b; t += SCAN_THREADS) s += sums[t];
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) lw[threadIdx.x >> 6] = s;
  __syncthreads();
  T add = 0;
#pragma unroll
  for (int i = 0; i < SCAN_THREADS / 64; ++i) add += lw[i];
  const uint64_t base = (uint64_t)b * SCAN_TILE;
  if (add)
    for (int i = threadIdx.x; i < SCAN_TILE; i += SCAN_THREADS)
      if (base + i < n) out[base + i] += add;
  if (total && b == tiles - 1 && threadIdx.x == 0) *total = add + sums[b];
}

// Scratch needed by scan_exclusive for n elements (bytes).
inline size_t scan_scratch_bytes(uint64_t n, size_t elem) {
  size_t b = 0;
  while (n > 1) {
    n = (n + SCAN_TILE - 1) / SCAN_TILE;
    b += ((n + 1) * elem + 63) / 64 * 64 + 64;
  }
  return b + 128;
}

// out[i] = sum_{j<i} in[i]; in == out allowed.  If total != nullptr, *total (device)
// receives the sum of all n inputs.  scratch: scan_scratch_bytes(n) bytes.
// small_ok = false: never the one-block k_scan_small (the nested scan of a large scan's tile
// sums, which may run beside the leaf kernel: a 1024-thread block waits for a whole CU to
// drain there -- the topology stream of a 100M build lost 6 ms to it).
// n_dev (nullable): a device-side count that caps n (a grid sized by the host's bound; the
// entries past the count are neither read nor written).
template <typename T>
void scan_exclusive(const T* in, T* out, uint64_t n, T* total, void* scratch, hipStream_t st, bool small_ok = true,
                    const uint32_t* n_dev = nullptr) {
  if (n == 0) {
    if (total) (void)hipMemsetAsync(total, 0, sizeof(T), st);
    return;
  }
  if (small_ok && !n_dev && n <= SCAN_SMALL_MAX) {
    hipLaunchKernelGGL(k_scan_small<T>, dim3(1), dim3(SCAN_SMALL_THREADS), 0, st, in, out, n, total);
    return;
  }
  uint64_t tiles = (n + SCAN_TILE - 1) / SCAN_TILE;
  // the last input element is kept by the tile that reads it (in == out allowed)
  T* sums = (T*)scratch;
  T* last_in = sums + tiles;  // one slot after the tile sums
  if (tiles <= SCAN_TWO_MAX_TILES) {
    hipLaunchKernelGGL(k_scan_tiles<T>, dim3((unsigned)tiles), dim3(SCAN_THREADS), 0, st, in, out, n, sums,
                       (T*)nullptr, n_dev);
    hipLaunchKernelGGL(k_scan_add_sums<T>, dim3((unsigned)tiles), dim3(SCAN_THREADS), 0, st, out, n, (const T*)sums,
                       (uint32_t)tiles, total, n_dev);
    return;
  }
  hipLaunchKernelGGL(k_scan_tiles<T>, dim3((unsigned)tiles), dim3(SCAN_THREADS), 0, st, in, out, n, sums,
                     total ? last_in : (T*)nullptr, n_dev);
  if (tiles > 1) {
    char* next = (char*)scratch + (((tiles + 1) * sizeof(T) + 63) / 64) * 64 + 64;
    scan_exclusive<T>(sums, sums, tiles, (T*)nullptr, next, st, false);
    hipLaunchKernelGGL(k_scan_add<T>, dim3((unsigned)tiles), dim3(SCAN_THREADS), 0, st, out, n, (const T*)sums,
                       n_dev);
  }
  if (total)
    hipLaunchKernelGGL(k_scan_total<T>, dim3(1), dim3(1), 0, st, (const T*)last_in, (const T*)out, n, total, n_dev);
}

// ---------------------------------------------------------------------------
// Radix sort of (key, uint32 val) pairs on key bits [lo_bit, hi_bit); keys are uint64
// (composite segment | key prefixes) or uint32 (the plain path's 32-bit key prefixes:
// 8 bytes a pair moved per pass instead of 12).  One sweep per pass: one launch counts the
// digits of every pass at once (a pass's digit totals do not depend on the order the earlier
// passes leave), then each pass is one launch whose tiles rank their keys, publish their digit
// counts and take the counts of the tiles before them by decoupled look-back.  (Each pass had
// been a histogram launch, a scan of the tiles x 256 counts unless the sort was small, and the
// scatter: 2 to 5 launches.)
// ---------------------------------------------------------------------------
constexpr int RS_THREADS = 256;
// 16 keys per thread: 4096-key tiles, so a digit's run in a tile averages 16 keys (64 B
// of 32-bit prefixes) per store burst.  Measured at 100M (profiles/r2zc_sched_ab_100m.json):
// 4.52 ms for the plain-path sort against 5.03 ms with 2048-key tiles and 5.35 ms with 8192.
#ifndef KHST_RS_ITEMS
#define KHST_RS_ITEMS 16
#endif
constexpr int RS_ITEMS = KHST_RS_ITEMS;
constexpr int RS_TILE = RS_THREADS * RS_ITEMS;  // 4096 keys: 36 KiB of LDS staging (32-bit keys)
constexpr int RS_WAVES = RS_THREADS / 64;
constexpr int RS_MAX_PASSES = 8;
// Status word of (pass, tile, digit): bits 63:62 are 0 until the tile publishes, 1 for the
// tile's own count of the digit, 2 for the count over this tile and every tile before it;
// bits 61:0 hold the count.
constexpr unsigned long long RS_ST_AGG = 1ull << 62, RS_ST_INC = 2ull << 62, RS_ST_CNT = RS_ST_AGG - 1;
// scratch header: the digit totals of every pass, then the passes' tile tickets
constexpr size_t RS_HDR_BYTES = (RS_MAX_PASSES * 256 + RS_MAX_PASSES) * sizeof(uint32_t);
constexpr size_t RS_HDR_PAD = (RS_HDR_BYTES + 255) / 256 * 256;

// Digit totals of npass passes (bits lo_bit + 8p .. + 8) over all n keys, added into ghist
// (zeroed), and the first pass's status words cleared.  Grid-stride over tiles.
template <typename K, int IT>
__global__ void __launch_bounds__(RS_THREADS) k_rs_hist_all(const K* keys, uint64_t n, int lo_bit, int npass,
                                                            uint32_t* ghist, unsigned long long* st0, uint64_t nst) {
  constexpr int TILE = RS_THREADS * IT;
  __shared__ uint32_t h[RS_MAX_PASSES][256];
  for (int i = threadIdx.x; i < RS_MAX_PASSES * 256; i += RS_THREADS) (&h[0][0])[i] = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * RS_THREADS + threadIdx.x; i < nst; i += (uint64_t)gridDim.x * RS_THREADS)
    st0[i] = 0;
  __syncthreads();
  for (uint64_t t0 = (uint64_t)blockIdx.x * TILE; t0 < n; t0 += (uint64_t)gridDim.x * TILE) {
    // every key of the tile loaded before the first LDS atomic (the atomics would otherwise
    // hold each load back to its own round trip)
    K kk[IT];
#pragma unroll
    for (int it = 0; it < IT; ++it) {
      const uint64_t i = t0 + (uint64_t)it * RS_THREADS + threadIdx.x;
      kk[it] = keys[i < n ? i : n - 1];
    }
#pragma unroll
    for (int it = 0; it < IT; ++it) {
      if (t0 + (uint64_t)it * RS_THREADS + threadIdx.x < n)
        for (int p = 0; p < npass; ++p) atomicAdd(&h[p][(uint32_t)(kk[it] >> (lo_bit + 8 * p)) & 0xFF], 1u);
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < npass * 256; i += RS_THREADS) {
    const uint32_t v = (&h[0][0])[i];
    if (v) atomicAdd(&ghist[i], v);
  }
}

// One pass.  The tile index comes from a ticket (tiles are taken in launch order, so every
// tile a look-back waits for is already running).  Keys are ranked per wave (ballot
// multisplit), the tile's digit counts published, the counts of the tiles before it looked
// back for, the tile placed in LDS in digit order and written out so that each digit's run of
// the tile goes to consecutive global addresses (coalesced stores instead of one scattered
// store per key).  status_next (nullable): the next pass's status words, cleared here.
template <typename K, int IT = RS_ITEMS>
__global__ void __launch_bounds__(RS_THREADS) k_rs_pass(const K* keys, const uint32_t* vals, K* okeys,
                                                        uint32_t* ovals, uint64_t n, int shift, const uint32_t* ghist,
                                                        unsigned long long* status, unsigned long long* status_next,
                                                        uint32_t* ticket) {
  constexpr int TILE = RS_THREADS * IT, WSLICE = TILE / RS_WAVES;
  __shared__ uint32_t wc[RS_WAVES][256];
  __shared__ uint32_t tstart[256], gbase[256];
  __shared__ uint32_t lw[RS_THREADS / 64];
  __shared__ uint32_t s_tile;
  __shared__ K sk[TILE];
  __shared__ uint32_t sv[TILE];
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  if (threadIdx.x == 0) s_tile = atomicAdd(ticket, 1u);
  const uint32_t gtot = ghist[threadIdx.x];  // digit threadIdx.x over all tiles (RS_THREADS == 256 digits)
  if (status_next) status_next[(uint64_t)blockIdx.x * 256 + threadIdx.x] = 0;
  for (int i = threadIdx.x; i < RS_WAVES * 256; i += RS_THREADS) (&wc[0][0])[i] = 0;
  __syncthreads();
  const uint32_t tile = s_tile;
  const uint64_t tbase = (uint64_t)tile * TILE;
  const uint64_t base = tbase + (uint64_t)w * WSLICE;
  K k[IT];
  uint32_t v[IT];
  uint32_t r[IT];
  const uint64_t lt = lanemask_lt();
  // the whole slice loaded first: the ranking's LDS traffic and wave barriers would otherwise
  // hold each load back to its own HBM round trip (16 in a row per tile)
#pragma unroll
  for (int it = 0; it < IT; ++it) {
    uint64_t i = base + (uint64_t)it * 64 + lane;
    bool valid = i < n;
    k[it] = valid ? keys[i] : 0;
    v[it] = valid ? vals[i] : 0;
  }
#pragma unroll
  for (int it = 0; it < IT; ++it) {
    uint64_t i = base + (uint64_t)it * 64 + lane;
    bool valid = i < n;
    uint32_t d = (uint32_t)(k[it] >> shift) & 0xFF;
    uint64_t peers = __ballot(valid);
#pragma unroll
    for (int b = 0; b < 8; ++b) {
      bool bit = (d >> b) & 1;
      uint64_t bb = __ballot(bit);
      peers &= bit ? bb : ~bb;
    }
    uint32_t cnt = valid ? wc[w][d] : 0;
    uint32_t below = (uint32_t)__popcll(peers & lt);
    r[it] = cnt + below;
    // the lowest lane of each peer group bumps the wave's digit counter
    if (valid && below == 0) wc[w][d] = cnt + (uint32_t)__popcll(peers);
    __builtin_amdgcn_wave_barrier();
  }
  __syncthreads();
  // per digit: wave offsets inside the tile's digit run, the count published, tile-local run
  // start, the digit's global start, the count in earlier tiles (look-back)
  {
    const int d = threadIdx.x;
    uint32_t run = 0;
#pragma unroll
    for (int q = 0; q < RS_WAVES; ++q) {
      uint32_t t = wc[q][d];
      wc[q][d] = run;
      run += t;
    }
    unsigned long long* my = status + (uint64_t)tile * 256 + d;
    __hip_atomic_store(my, (tile == 0 ? RS_ST_INC : RS_ST_AGG) | run, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    uint32_t tot;
    tstart[d] = block_exclusive_scan<uint32_t>(run, lw, &tot);
    const uint32_t dbase = block_exclusive_scan<uint32_t>(gtot, lw, &tot);
    uint64_t excl = 0;
    if (tile > 0) {
      for (uint64_t t = tile - 1;;) {
        const unsigned long long s =
            __hip_atomic_load(status + t * 256 + d, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if ((s >> 62) == 0) {  // not published yet (its tile is running: it took an earlier ticket)
          __builtin_amdgcn_s_sleep(1);
          continue;
        }
        excl += s & RS_ST_CNT;
        if ((s >> 62) == 2) break;  // (tile 0 publishes its count as inclusive)
        --t;
      }
      __hip_atomic_store(my, RS_ST_INC | (excl + run), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    gbase[d] = dbase + (uint32_t)excl;
  }
  __syncthreads();
#pragma unroll
  for (int it = 0; it < IT; ++it) {
    uint64_t i = base + (uint64_t)it * 64 + lane;
    if (i < n) {
      uint32_t d = (uint32_t)(k[it] >> shift) & 0xFF;
      uint32_t li = tstart[d] + wc[w][d] + r[it];
      sk[li] = k[it];
      sv[li] = v[it];
    }
  }
  __syncthreads();
  const uint32_t tn = (uint32_t)((n - tbase) < (uint64_t)TILE ? (n - tbase) : (uint64_t)TILE);
  for (uint32_t li = threadIdx.x; li < tn; li += RS_THREADS) {
    K key = sk[li];
    uint32_t d = (uint32_t)(key >> shift) & 0xFF;
    uint32_t pos = gbase[d] + (li - tstart[d]);
    okeys[pos] = key;
    ovals[pos] = sv[li];
  }
}

// Small sorts (a block commit's ops and elements, up to RS_SMALL_N keys) take 1024-key tiles
// (4 keys per thread): 4x the blocks, a quarter of each block's serial ranking -- the passes
// are latency-bound at these sizes.
constexpr int RS_SMALL_ITEMS = 4;
constexpr uint64_t RS_SMALL_N = 65536;
// Large sorts (from RS_BIG_N keys: a full build's) take RS_BIG_ITEMS keys per thread: with the
// one-sweep passes fewer, longer tiles publish and look back less and store longer digit runs
// (100M: the 4 passes 3.40 -> 3.00 ms with 8192-key tiles, profiles/r6k_radix_tile_ab_100m.json)
// at 2 waves per SIMD; below RS_BIG_N they would leave CUs without a tile.
#ifndef KHST_RS_BIG_ITEMS
#define KHST_RS_BIG_ITEMS 32
#endif
constexpr int RS_BIG_ITEMS = KHST_RS_BIG_ITEMS;
constexpr uint64_t RS_BIG_N = 1ull << 22;
// (the big tiles for 32-bit keys only: 64-bit ones would hold 101 KB of LDS a block)
inline int radix_items(uint64_t n, size_t key_bytes) {
  return n <= RS_SMALL_N ? RS_SMALL_ITEMS : (n >= RS_BIG_N && key_bytes == 4) ? RS_BIG_ITEMS : RS_ITEMS;
}
inline uint64_t radix_tiles(uint64_t n, size_t key_bytes) {
  const uint64_t tile = (uint64_t)RS_THREADS * (uint64_t)radix_items(n, key_bytes);
  return (n + tile - 1) / tile;
}
inline size_t radix_scratch_bytes(uint64_t n) {  // (64-bit keys: the most tiles)
  return RS_HDR_PAD + 2 * radix_tiles(n, 8) * 256 * sizeof(unsigned long long) + 256;
}

// Sorts (k0, v0) on bits [lo_bit, hi_bit) (multiples of 8, at most 64 bits), using (k1, v1)
// as ping-pong buffers.  Returns true if the result ended in (k1, v1).  n must be < 2^32.
// Launches: a fill of the scratch header, the digit count, one per pass.
// hdr_zeroed: the caller's previous kernel zeroed the scratch header (RS_HDR_BYTES): no fill launch
template <typename K>
inline bool radix_sort_pairs(K* k0, uint32_t* v0, K* k1, uint32_t* v1, uint64_t n, int lo_bit, int hi_bit,
                             void* scratch, hipStream_t st, bool hdr_zeroed = false) {
  if (n <= 1 || hi_bit <= lo_bit) return false;
  const int items = radix_items(n, sizeof(K));
  const uint64_t tiles = radix_tiles(n, sizeof(K));
  const int npass = (hi_bit - lo_bit + 7) / 8;
  uint32_t* ghist = (uint32_t*)scratch;
  uint32_t* ticket = ghist + RS_MAX_PASSES * 256;
  unsigned long long* stat[2] = {(unsigned long long*)((char*)scratch + RS_HDR_PAD), nullptr};
  stat[1] = stat[0] + tiles * 256;
  if (!hdr_zeroed) (void)hipMemsetAsync(ghist, 0, RS_HDR_BYTES, st);
  const unsigned hgrid = (unsigned)(tiles < 1024 ? tiles : 1024);
  // (the digit count's tile is only its loop step: large sorts take RS_ITEMS keys per thread)
  if (items == RS_SMALL_ITEMS)
    hipLaunchKernelGGL((k_rs_hist_all<K, RS_SMALL_ITEMS>), dim3(hgrid), dim3(RS_THREADS), 0, st, (const K*)k0, n,
                       lo_bit, npass, ghist, stat[0], tiles * 256);
  else
    hipLaunchKernelGGL((k_rs_hist_all<K, RS_ITEMS>), dim3(hgrid), dim3(RS_THREADS), 0, st, (const K*)k0, n, lo_bit,
                       npass, ghist, stat[0], tiles * 256);
  bool flip = false;
  for (int p = 0; p < npass; ++p) {
    K* ik = flip ? k1 : k0;
    uint32_t* iv = flip ? v1 : v0;
    K* ok = flip ? k0 : k1;
    uint32_t* ov = flip ? v0 : v1;
    unsigned long long* nxt = p + 1 < npass ? stat[(p + 1) & 1] : nullptr;
    if (items == RS_SMALL_ITEMS)
      hipLaunchKernelGGL((k_rs_pass<K, RS_SMALL_ITEMS>), dim3((unsigned)tiles), dim3(RS_THREADS), 0, st, (const K*)ik,
                         (const uint32_t*)iv, ok, ov, n, lo_bit + 8 * p, (const uint32_t*)(ghist + 256 * p), stat[p & 1],
                         nxt, ticket + p);
    else if (sizeof(K) == 4 && items == RS_BIG_ITEMS)
      hipLaunchKernelGGL((k_rs_pass<K, sizeof(K) == 4 ? RS_BIG_ITEMS : RS_ITEMS>), dim3((unsigned)tiles), dim3(RS_THREADS), 0, st, (const K*)ik,
                         (const uint32_t*)iv, ok, ov, n, lo_bit + 8 * p, (const uint32_t*)(ghist + 256 * p), stat[p & 1],
                         nxt, ticket + p);
    else
      hipLaunchKernelGGL((k_rs_pass<K>), dim3((unsigned)tiles), dim3(RS_THREADS), 0, st, (const K*)ik,
                         (const uint32_t*)iv, ok, ov, n, lo_bit + 8 * p, (const uint32_t*)(ghist + 256 * p), stat[p & 1],
                         nxt, ticket + p);
    flip = !flip;
  }
  return flip;
}

}  // namespace khst
