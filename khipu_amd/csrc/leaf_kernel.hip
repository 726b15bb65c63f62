// k_leaf_in, the early-leaf kernel of plain root builds (the dominant kernel of the 100M step),
// in a compilation unit of its own so that it is compiled without -falign-loops=64, which the
// rest of the library takes (khst.hip).  The VALU-bound kernels here are sensitive to code
// placement: aligning the loop heads to 64 bytes took key hashing 11.4 -> 10.3 ms and the
// branch levels 8.3 -> 7.6 ms at 100M, but this kernel 13.5 -> 14.8 ms (the 64-byte alignment
// of its 4-run loop moves its 41-KB straight-line permutation; same box, alternating runs,
// profiles/r8i_align_ab_100m.json).  Nothing else differs: the kernel's code is as it was.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "keccak.h"
#include "trie_ops.h"
#include "wave.h"

using namespace khst;

namespace {
constexpr int BS = 256;
constexpr uint32_t LEAF_ITEMS = 4;  // (khst.hip sizes the grid with the same value)
}  // namespace

// Early leaves (plain root builds; trie_ops.h op_leaf_core): one thread per INPUT, on the
// second stream beside the branch topology.  Keys and packed values are read in input
// order; the parent depth gives the header geometry, the key and value are then loaded at
// their message shifts, and the message is assembled dword by dword (v_perm_b32) straight
// into the Keccak state.  Every lane of a wave runs the wave-bound reductions, so threads
// past n take part with neutral values.
// A block takes LEAF_ITEMS runs of BS consecutive inputs, one after the other: the next run's
// scatter record and span offsets (the first of the two dependent load rounds) are brought
// into LDS by LDS-DMA while the current input is assembled and permuted (no registers held
// across the permutation), and the counters are added once per wave (42.6 -> 41.9 ms in the
// step against one input per thread, profiles/r5g_leaf_prefetch_ab_100m.json).  Blocks that
// live for a few runs only keep the wave slots turning over for the topology kernels beside
// them (a persistent grid starved them: the topology stream 15 -> 22 ms, the step 42.5 -> 45
// ms, profiles/r5e_leaf_grid_ab_100m.json; forcing 7 waves per SIMD spilled and cost 1.4 ms).
// The permutation is straight-line (keccakf<KECCAK_FULL>: no pi-renaming moves at loop
// back-edges; 78 VGPRs and 6 waves with the 3-iteration loop, 0.9 ms slower in the step,
// profiles/r4bp_keccak_unroll_ab_100m.json).
// KH_LEAF_SHIFT (measurement builds): N s_nops at the kernel's entry move all of its code by 4N bytes
#if defined(KH_LEAF_SHIFT)
#define KH_STR2(x) #x
#define KH_STR(x) KH_STR2(x)
#define KH_LEAF_ENTRY() asm volatile(".rept " KH_STR(KH_LEAF_SHIFT) "\n\ts_nop 0\n\t.endr")
#else
#define KH_LEAF_ENTRY() ((void)0)
#endif
__global__ void __launch_bounds__(BS) k_leaf_in(Topo T, uint64_t n) {
  KH_LEAF_ENTRY();
  auto wave = [](bool use, uint32_t e, uint32_t llo, uint32_t lhi) {
    WaveBounds b;
    b.emax = wave_max_u32(use ? e : 0u);
    b.emin = 255u - wave_max_u32(use ? 255u - e : 0u);
    b.Lmax = wave_max_u32(use ? lhi : 0u);
    b.Lmin = 255u - wave_max_u32(use ? 255u - llo : 0u);
    return b;
  };
  const uint64_t j0 = (uint64_t)blockIdx.x * LEAF_ITEMS * BS + threadIdx.x, jend = j0 + LEAF_ITEMS * BS;
  // double-buffered per wave: [slot][wave][pv low / pv high dwords (2 x 64), voff[j], voff[j+1] (64 pairs)]
  __shared__ uint32_t pbuf[2][BS / 64][64 * 6];
  const uint32_t w = threadIdx.x >> 6, l = threadIdx.x & 63;
  auto issue = [&](uint32_t slot, uint64_t j) {  // (every lane of the wave: j past n reads a clamped input)
    typedef __attribute__((address_space(1))) void gv;
    typedef __attribute__((address_space(3))) void lv;
    const uint64_t jj = j < n ? j : n - 1;
    uint32_t* b = pbuf[slot][w];
    __builtin_amdgcn_global_load_lds((gv*)(T.pdinv + jj), (lv*)b, 4, 0, 0);
    __builtin_amdgcn_global_load_lds((gv*)((const uint32_t*)(T.pdinv + jj) + 1), (lv*)(b + 64), 4, 0, 0);
    __builtin_amdgcn_global_load_lds((gv*)(T.voff + jj), (lv*)(b + 128), 16, 0, 0);
  };
  auto take = [&](uint32_t slot, uint64_t j, uint64_t& pv, uint64_t& off, uint64_t& end) {
    __builtin_amdgcn_s_waitcnt(0);  // (vmcnt: the slot's LDS-DMA has landed)
    asm volatile("" ::: "memory");
    const uint32_t* b = pbuf[slot][w];
    pv = j < n ? ((uint64_t)b[64 + l] << 32) | b[l] : PDINV_SKIP;
    off = ((const uint64_t*)(b + 128))[2 * l];
    end = ((const uint64_t*)(b + 128))[2 * l + 1];
  };
  const uintptr_t vend = (uintptr_t)T.vals + T.voff[n];  // (once: see op_leaf_core)
  uint64_t pv = 0, off = 0, end = 0;
  issue(0, j0);
  uint32_t perms = 0, inl = 0, slot = 0;
#pragma unroll 1
  for (uint64_t j = j0; j < jend && j - threadIdx.x % 64 < n; j += BS) {  // (wave-uniform: the wave's first input)
    const uint64_t jn = j + BS < jend ? j + BS : n;
    take(slot, j, pv, off, end);
    if (j + BS < jend && jn - threadIdx.x % 64 < n) issue(slot ^ 1, jn);  // (wave-uniform: no next run past the block's)
    slot ^= 1;
    const bool live = pv != PDINV_SKIP;  // not an earlier put of a key put again later
    uint32_t in1 = 0, lb = 0;
    perms += op_leaf_core(T, live, (int32_t)(int8_t)(uint8_t)(pv >> 32), (uint32_t)pv, j, n, off,
                          (uint32_t)(end - off), vend, wave, &in1, &lb);
    inl += in1;
    if (lb) atomicAdd(&T.ctr[CTR_LONGB], (unsigned long long)lb);
  }
  const unsigned long long sp = wave_sum((unsigned long long)perms), si = wave_sum((unsigned long long)inl);
  if ((threadIdx.x & 63) == 0) {
    if (sp) {
      atomicAdd(ctr_stat(T.ctr, CTR_PERMS, blockIdx.x), sp);
      atomicAdd(ctr_stat(T.ctr, CTR_HASHES, blockIdx.x), sp);
    }
    if (si) atomicAdd(ctr_stat(T.ctr, CTR_INLINE, blockIdx.x), si);
  }
}
