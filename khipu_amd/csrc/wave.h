// Wave-level device helpers (64-lane wavefronts): DPP / shuffle reductions, per-wave counter
// claims, and the topology kernels' issue priority.  Included by prims.h and by the early-leaf
// kernel's compilation unit (leaf_kernel.hip), which takes nothing else from prims.h.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace khst {

constexpr int WAVE = 64;

// Issue priority of the latency-bound topology kernels that run beside the VALU-bound leaf
// kernel (scans, pyramid, list kernels, branch records, level order): s_setprio raises their
// waves over the leaf waves in the SIMD's issue arbitration (priority, then age), so a long-
// lived leaf wave does not win every issue slot from a younger topology wave.
__device__ __forceinline__ void topo_prio() { __builtin_amdgcn_s_setprio(2); }

// max over the wave's 64 lanes (DPP row shifts + row broadcasts), returned to every lane
__device__ __forceinline__ uint32_t wave_max_u32(uint32_t v) {
  v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xF, 0xF, true));  // row_shr:1
  v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xF, 0xF, true));  // row_shr:2
  v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xF, 0xF, true));  // row_shr:4
  v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xF, 0xF, true));  // row_shr:8
  v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xA, 0xF, false));  // row_bcast:15
  v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xC, 0xF, false));  // row_bcast:31
  return (uint32_t)__builtin_amdgcn_readlane((int)v, 63);
}
__device__ __forceinline__ uint64_t lanemask_lt() {
  uint32_t lane = __lane_id();
  return lane == 0 ? 0ULL : (~0ULL >> (64 - lane));
}

// One atomicAdd per wave: the active lanes with `want` get consecutive slots of *ctr (a
// counter shared by a whole grid would otherwise serialise one atomic per lane).  Every
// active lane must call it (divergent paths aggregate among their own lanes).
__device__ __forceinline__ uint64_t wave_claim(unsigned long long* ctr, bool want) {
  const uint64_t m = __ballot(want);
  if (m == 0) return 0;
  const int leader = __ffsll((long long)m) - 1;
  unsigned long long base = 0;
  if ((int)__lane_id() == leader) base = atomicAdd(ctr, (unsigned long long)__popcll(m));
  const uint32_t lo = (uint32_t)__shfl((int)(uint32_t)base, leader);
  const uint32_t hi = (uint32_t)__shfl((int)(uint32_t)(base >> 32), leader);
  return (((uint64_t)hi << 32) | lo) + (uint64_t)__popcll(m & lanemask_lt());
}

template <typename T>
__device__ __forceinline__ T wave_sum(T v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

// add v (per lane) into *dst with one atomic per wave
__device__ __forceinline__ void wave_atomic_add(unsigned long long* dst, unsigned long long v) {
  v = wave_sum(v);
  if (__lane_id() == 0 && v) atomicAdd(dst, v);
}

}  // namespace khst
