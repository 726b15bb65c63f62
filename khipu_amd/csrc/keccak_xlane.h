// Keccak-f[1600] spread over the lanes of a 32-lane group (N1, "DPP / cross-lane where that
// beats one thread per node"): for the latency-bound small levels of a block commit.
//
// One thread per node runs the whole permutation alone: ~4,400 dependent VALU
// instructions, ~9 us when its wave has the SIMD to itself (a level of a few thousand
// branches; scripts/xlane_check.hip).  Here lane sub = x + 5y (0..24) of the group holds
// state lane A[x, y] as two 32-bit halves, and a round is
//   1. A -> LDS;  lane (X, Y) reads its pi source A[x, y] (x = 3(Y - 3X), y = X, mod 5) and
//      the columns x - 1 and x + 1, forms theta's A ^ C[x-1] ^ rot(C[x+1], 1) and rotates it
//      by rho[x, y]: B[X, Y]                                             (xl_step_theta_rho)
//   2. B -> LDS;  chi from B[X+1, Y] and B[X+2, Y]; iota on lane 0        (xl_step_chi)
// ~22 VALU and two LDS round trips per round instead of 180 VALU.  A wave's LDS operations
// execute in order, so the group needs no barrier, only the compiler fences of xl_sync().
// Lanes 25..31 compute on their own LDS slots (the buffers are 32 words) and are ignored.
// The two steps are host + device code: tests/emu replays them lane by lane against the
// one-thread permutation.  Reference behaviour: KeccakCore.scala:103-531 (as keccak.h).
#pragma once
#include "keccak.h"

namespace khst {

struct XLane {
  uint32_t sub;     // this lane's state index (x + 5y), or 25..31
  uint32_t src;     // pi source of B[sub]
  uint32_t cm, cp;  // first index of the columns x - 1 and x + 1 of the source
  uint32_t n1, n2;  // chi neighbours (X + 1, Y), (X + 2, Y)
  uint32_t rsh;     // rho of the source as a funnel shift (see xl_step_theta_rho)
  bool rswap;       //   and whether the halves swap first
  bool iota;        // lane 0
};

KH_HD XLane xlane_setup(uint32_t sub) {
  constexpr uint8_t ROT[25] = {0, 1, 62, 28, 27, 36, 44, 6, 55, 20, 3, 10, 43, 25, 39, 41, 45, 15, 21, 8, 18, 2, 61, 56, 14};
  XLane g;
  g.sub = sub;
  const uint32_t s = sub < 25 ? sub : 0;  // lanes past the state read valid slots
  const uint32_t X = s % 5, Y = s / 5;
  const uint32_t sy = X, sx = (3 * (Y + 15 - 3 * X)) % 5;
  g.src = sx + 5 * sy;
  g.cm = (sx + 4) % 5;
  g.cp = (sx + 1) % 5;
  g.n1 = (X + 1) % 5 + 5 * Y;
  g.n2 = (X + 2) % 5 + 5 * Y;
  // rotl64 by r = ROT[src]: swap the halves when r >= 32 (and for r == 0), then one funnel
  // shift by (32 - r) & 31 per half (r == 0: swapped halves shifted by 0 = the identity)
  const uint32_t r = ROT[g.src];
  g.rswap = r == 0 || r >= 32;
  g.rsh = (32 - (r & 31)) & 31;
  g.iota = sub == 0;
  return g;
}

// low 32 bits of ({a, b} >> (s & 31)): v_alignbit_b32 (a shift of 0 gives b)
KH_HD uint32_t funnel0(uint32_t a, uint32_t b, uint32_t s) {
#ifdef __HIP_DEVICE_COMPILE__
  return __builtin_amdgcn_alignbit(a, b, s);
#else
  return (uint32_t)((((uint64_t)a << 32) | b) >> (s & 31));
#endif
}

// step 1 of a round for lane g: B[sub] from the state A (every lane's word, in bA)
KH_HD uint64_t xl_step_theta_rho(const XLane& g, const uint64_t* bA) {
  const uint64_t a = bA[g.src];
  const uint64_t m0 = bA[g.cm], m1 = bA[g.cm + 5], m2 = bA[g.cm + 10], m3 = bA[g.cm + 15], m4 = bA[g.cm + 20];
  const uint64_t p0 = bA[g.cp], p1 = bA[g.cp + 5], p2 = bA[g.cp + 10], p3 = bA[g.cp + 15], p4 = bA[g.cp + 20];
  const uint32_t c1l = xor3(xor3((uint32_t)m0, (uint32_t)m1, (uint32_t)m2), (uint32_t)m3, (uint32_t)m4);
  const uint32_t c1h = xor3(xor3((uint32_t)(m0 >> 32), (uint32_t)(m1 >> 32), (uint32_t)(m2 >> 32)),
                            (uint32_t)(m3 >> 32), (uint32_t)(m4 >> 32));
  const uint32_t c2l = xor3(xor3((uint32_t)p0, (uint32_t)p1, (uint32_t)p2), (uint32_t)p3, (uint32_t)p4);
  const uint32_t c2h = xor3(xor3((uint32_t)(p0 >> 32), (uint32_t)(p1 >> 32), (uint32_t)(p2 >> 32)),
                            (uint32_t)(p3 >> 32), (uint32_t)(p4 >> 32));
  // theta: a ^ C[x-1] ^ rot(C[x+1], 1)
  const uint32_t tl = xor3((uint32_t)a, c1l, funnel(c2l, c2h, 31));
  const uint32_t th = xor3((uint32_t)(a >> 32), c1h, funnel(c2h, c2l, 31));
  // rho (per-lane amount); the result lands at the pi destination = this lane
  const uint32_t h0 = g.rswap ? tl : th, l0 = g.rswap ? th : tl;
  const uint32_t bh = funnel0(h0, l0, g.rsh);
  const uint32_t bl = funnel0(l0, h0, g.rsh);
  return ((uint64_t)bh << 32) | bl;
}

// step 2: chi from this lane's B and its row neighbours in bB, iota on lane 0
KH_HD uint64_t xl_step_chi(const XLane& g, uint64_t b, const uint64_t* bB, int rd) {
  const uint64_t b1 = bB[g.n1], b2 = bB[g.n2];
  const uint64_t rc = g.iota ? round_constant(rd) : 0;
  return (b ^ (~b1 & b2)) ^ rc;
}

#ifdef __HIPCC__
__device__ __forceinline__ void xl_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// buf: the group's 64 words of LDS (two 32-word buffers)
__device__ __forceinline__ void keccakf_xlane(uint32_t& lo, uint32_t& hi, uint64_t* buf, const XLane& g) {
  uint64_t* bA = buf;
  uint64_t* bB = buf + 32;
  uint64_t a = ((uint64_t)hi << 32) | lo;
#pragma unroll 2
  for (int rd = 0; rd < 24; ++rd) {
    bA[g.sub] = a;
    xl_sync();
    const uint64_t b = xl_step_theta_rho(g, bA);
    bB[g.sub] = b;
    xl_sync();
    a = xl_step_chi(g, b, bB, rd);
  }
  lo = (uint32_t)a;
  hi = (uint32_t)(a >> 32);
}
#endif

}  // namespace khst
