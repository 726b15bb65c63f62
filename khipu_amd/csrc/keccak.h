// Keccak-256 (legacy 0x01 padding) for gfx950: one message per lane, the 25-lane
// Keccak-f[1600] state held in 50 VGPRs (25 lanes x 32-bit halves).
//
// Reference behaviour: khipu-base/.../crypto/hash/KeccakCore.scala:39-52 (RC),
// :103-531 (processBlock), :534-562 (doPadding: 0x01 .. 0x80, 0x81 if one byte
// is left), :570 (rate 136 B); DigestEngine.scala:102-166 (a block is absorbed
// as soon as 136 bytes are buffered, so L bytes cost floor(L/136)+1 permutations).
//
// gfx950's VALU is 32-bit: the permutation is written on 32-bit halves so that
// theta's 5-way XOR becomes v_xor3_b32 pairs, every 64-bit rotate two
// v_alignbit_b32 (funnel shifts); gfx950's v_bitop3_b32 does theta's 3-way XORs (the
// column parities, and A ^ C[x-1] ^ rot(C[x+1], 1) in one step: D is never formed) and
// chi's a ^ (~b & c) in one instruction each: 180 VALU ops per round (120 v_bitop3,
// 58 v_alignbit, iota) against the canonical 240 of SURVEY §8d (which assumes v_xor3 +
// v_bfi + v_xor).  Every state index is a
// compile-time constant after unrolling, so the state never leaves registers.
#pragma once
#include <stdint.h>
#ifdef __HIPCC__
#include <hip/hip_runtime.h>
#define KH_HD __host__ __device__ __forceinline__
#else  // host-only compilation of the same code (tests/emu)
#define KH_HD inline
#endif

namespace khst {

// Round constants.  The device reads its own __constant__ copy; host code (the
// root fold, tests/emu) reads a plain array: the host shadow of a __constant__
// variable is not the initialised table.
#ifdef __HIPCC__
__constant__ static const uint64_t kRC_dev[24] = {
    0x0000000000000001ULL, 0x0000000000008082ULL, 0x800000000000808AULL, 0x8000000080008000ULL,
    0x000000000000808BULL, 0x0000000080000001ULL, 0x8000000080008081ULL, 0x8000000000008009ULL,
    0x000000000000008AULL, 0x0000000000000088ULL, 0x0000000080008009ULL, 0x000000008000000AULL,
    0x000000008000808BULL, 0x800000000000008BULL, 0x8000000000008089ULL, 0x8000000000008003ULL,
    0x8000000000008002ULL, 0x8000000000000080ULL, 0x000000000000800AULL, 0x800000008000000AULL,
    0x8000000080008081ULL, 0x8000000000008080ULL, 0x0000000080000001ULL, 0x8000000080008008ULL};
#endif
static const uint64_t kRC_host[24] = {
    0x0000000000000001ULL, 0x0000000000008082ULL, 0x800000000000808AULL, 0x8000000080008000ULL,
    0x000000000000808BULL, 0x0000000080000001ULL, 0x8000000080008081ULL, 0x8000000000008009ULL,
    0x000000000000008AULL, 0x0000000000000088ULL, 0x0000000080008009ULL, 0x000000008000000AULL,
    0x000000008000808BULL, 0x800000000000008BULL, 0x8000000000008089ULL, 0x8000000000008003ULL,
    0x8000000000008002ULL, 0x8000000000000080ULL, 0x000000000000800AULL, 0x800000008000000AULL,
    0x8000000080008081ULL, 0x8000000000008080ULL, 0x0000000080000001ULL, 0x8000000080008008ULL};
KH_HD uint64_t round_constant(int r) {
#ifdef __HIP_DEVICE_COMPILE__
  return kRC_dev[r];
#else
  return kRC_host[r];
#endif
}

// 32-bit funnel shift: low 32 bits of ({a, b} >> s), s in [1, 31] -> v_alignbit_b32.
KH_HD uint32_t funnel(uint32_t a, uint32_t b, uint32_t s) {
#ifdef __HIP_DEVICE_COMPILE__
  return __builtin_amdgcn_alignbit(a, b, s);
#else
  return (uint32_t)((((uint64_t)a << 32) | b) >> s);
#endif
}

// a ^ b ^ c in one instruction (v_bitop3_b32, truth table 0x96) on gfx950.
KH_HD uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
#ifdef __HIP_DEVICE_COMPILE__
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
#else
  return a ^ b ^ c;
#endif
}

// rotate-left of the 64-bit lane (h:l) by n (a compile-time constant after unrolling)
KH_HD void rotl_hl(uint32_t& l, uint32_t& h, int n) {
  uint32_t nl, nh;
  if (n == 0) return;
  if (n < 32) {
    nh = funnel(h, l, 32 - n);
    nl = funnel(l, h, 32 - n);
  } else if (n == 32) {
    nh = l;
    nl = h;
  } else {
    nh = funnel(l, h, 64 - n);
    nl = funnel(h, l, 64 - n);
  }
  l = nl;
  h = nh;
}

struct KState {
  uint32_t lo[25], hi[25];
};

KH_HD void keccak_round(KState& S, uint64_t rc) {
  constexpr int ROT[25] = {0, 1, 62, 28, 27, 36, 44, 6, 55, 20, 3, 10, 43, 25, 39, 41, 45, 15, 21, 8, 18, 2, 61, 56, 14};
  uint32_t CL[5], CH[5], RL[5], RH[5], BL[25], BH[25];
#pragma unroll
  for (int x = 0; x < 5; ++x) {  // theta: column parities
    CL[x] = xor3(xor3(S.lo[x], S.lo[x + 5], S.lo[x + 10]), S.lo[x + 15], S.lo[x + 20]);
    CH[x] = xor3(xor3(S.hi[x], S.hi[x + 5], S.hi[x + 10]), S.hi[x + 15], S.hi[x + 20]);
  }
#pragma unroll
  for (int x = 0; x < 5; ++x) {  // rot(C[x], 1)
    uint32_t rl = CL[x], rh = CH[x];
    rotl_hl(rl, rh, 1);
    RL[x] = rl;
    RH[x] = rh;
  }
#pragma unroll
  for (int x = 0; x < 5; ++x)
#pragma unroll
    for (int y = 0; y < 5; ++y) {  // theta apply (A ^= C[x-1] ^ rot(C[x+1], 1): one v_bitop3 per
                                   // half, D is never formed), rho, pi
      const int i = x + 5 * y;
      uint32_t l = xor3(S.lo[i], CL[(x + 4) % 5], RL[(x + 1) % 5]);
      uint32_t h = xor3(S.hi[i], CH[(x + 4) % 5], RH[(x + 1) % 5]);
      rotl_hl(l, h, ROT[i]);
      const int d = y + 5 * ((2 * x + 3 * y) % 5);
      BL[d] = l;
      BH[d] = h;
    }
#pragma unroll
  for (int y = 0; y < 5; ++y)
#pragma unroll
    for (int x = 0; x < 5; ++x) {  // chi
      const int i = x + 5 * y, i1 = (x + 1) % 5 + 5 * y, i2 = (x + 2) % 5 + 5 * y;
      S.lo[i] = BL[i] ^ (~BL[i1] & BL[i2]);
      S.hi[i] = BH[i] ^ (~BH[i1] & BH[i2]);
    }
  S.lo[0] ^= (uint32_t)rc;  // iota
  S.hi[0] ^= (uint32_t)(rc >> 32);
}

// U rounds per loop iteration.  8 (3 iterations; the pi renaming costs ~5 moves per round, 42
// per back-edge) by default: the branch kernels inline several permutations, and at 24 their
// code outgrows the instruction cache (58 -> 129 KB; branch levels 1.0 ms longer at 100M).
// 24, straight-line, in the leaf kernel (op_leaf_core): no moves, 78 -> 69 VGPRs, 7 waves per
// SIMD, 15.6 -> 14.8 ms at 100M.  Key hashing measured no faster straight-line (8 waves per
// SIMD at 61 VGPRs; profiles/r4bp_keccak_unroll_ab_100m.json)
#ifndef KECCAK_LOOP_ROUNDS
#define KECCAK_LOOP_ROUNDS 8  // (measurement builds: -DKECCAK_LOOP_ROUNDS=24 unrolls every permutation)
#endif
constexpr int KECCAK_LOOP = KECCAK_LOOP_ROUNDS, KECCAK_FULL = 24;
template <int U = KECCAK_LOOP>
KH_HD void keccakf(KState& s) {
#pragma unroll U
  for (int r = 0; r < 24; ++r) keccak_round(s, round_constant(r));
}

KH_HD uint64_t lane(const KState& s, int i) { return ((uint64_t)s.hi[i] << 32) | s.lo[i]; }

// ---- Keccak-f on a lane pair (k_branch_small: levels of 8k-32k branches, a wave or two per
// SIMD, where one thread's permutation -- 180 dependent VALU a round at 4 cycles each -- is the
// level's latency).  Lane 2i holds the low halves of the 25 state words, lane 2i + 1 the high
// halves, in W[25].  Every 64-bit rotation becomes one DPP swap with the partner lane and one
// funnel shift, the same instruction on both lanes (low lane: (l, h) -> l' = {l:h} >> (32 - n);
// high lane: (h, l) -> h' = {h:l} >> (32 - n); past 32 the operands trade places); theta's
// parities and chi stay lane-local.  120 VALU a round per lane.  Both lanes of a pair must be
// active (the DPP reads the partner).
KH_HD uint32_t pair_partner(uint32_t x) {
#ifdef __HIP_DEVICE_COMPILE__
  // quad_perm [1,0,3,2]; bound_ctrl set, so no "old" operand is materialised (every lane reads
  // its partner: the v_mov of a zero old value before each DPP move was a fifth of the round)
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0xB1, 0xF, 0xF, true);
#else
  return x;  // (host code never runs the pair form)
#endif
}
KH_HD bool pair_odd() {
#ifdef __HIP_DEVICE_COMPILE__
  return __lane_id() & 1;
#else
  return false;
#endif
}
KH_HD uint32_t rotl_pair(uint32_t v, int n) {
  if (n == 0) return v;
  const uint32_t p = pair_partner(v);
  return n < 32 ? funnel(v, p, 32 - n) : n == 32 ? p : funnel(p, v, 64 - n);
}
KH_HD void keccak_round_pair(uint32_t* W, uint32_t rc_half) {
  constexpr int ROT[25] = {0, 1, 62, 28, 27, 36, 44, 6, 55, 20, 3, 10, 43, 25, 39, 41, 45, 15, 21, 8, 18, 2, 61, 56, 14};
  uint32_t C[5], R[5], B[25];
#pragma unroll
  for (int x = 0; x < 5; ++x) C[x] = xor3(xor3(W[x], W[x + 5], W[x + 10]), W[x + 15], W[x + 20]);
#pragma unroll
  for (int x = 0; x < 5; ++x) R[x] = funnel(C[x], pair_partner(C[x]), 31);  // this lane's half of rot(C[x], 1)
#pragma unroll
  for (int x = 0; x < 5; ++x)
#pragma unroll
    for (int y = 0; y < 5; ++y) {
      const int i = x + 5 * y;
      B[y + 5 * ((2 * x + 3 * y) % 5)] = rotl_pair(xor3(W[i], C[(x + 4) % 5], R[(x + 1) % 5]), ROT[i]);
    }
#pragma unroll
  for (int y = 0; y < 5; ++y)
#pragma unroll
    for (int x = 0; x < 5; ++x) {
      const int i = x + 5 * y;
      W[i] = B[i] ^ (~B[(x + 1) % 5 + 5 * y] & B[(x + 2) % 5 + 5 * y]);
    }
  W[0] ^= rc_half;
}
template <int U = KECCAK_LOOP>
KH_HD void keccakf_pair(uint32_t* W, bool odd) {
#pragma unroll U
  for (int r = 0; r < 24; ++r) {
    const uint64_t rc = round_constant(r);
    keccak_round_pair(W, odd ? (uint32_t)(rc >> 32) : (uint32_t)rc);
  }
}

// XOR word w into rate lane i (i compile-time after unrolling).
KH_HD void kxor(KState& s, int i, uint64_t w) {
  s.lo[i] ^= (uint32_t)w;
  s.hi[i] ^= (uint32_t)(w >> 32);
}

// nb (1..8) little-endian bytes from an arbitrary address via aligned 8-byte
// loads; only the aligned words holding bytes [p, p+nb) are read, so no access
// leaves the 8-byte-aligned span of the message.  Bytes above nb are garbage.
KH_HD uint64_t load64u_n(const uint8_t* p, uint32_t nb) {
  // pointer arithmetic, not an int round trip, so the address space survives (ds_read / global_load)
  uint32_t off = (uint32_t)((uintptr_t)p & 7);
  const uint64_t* q = (const uint64_t*)(p - off);
  uint64_t lo = q[0] >> (8 * off);
  if (off + nb > 8) lo |= q[1] << (64 - 8 * off);
  return lo;
}

KH_HD uint64_t low_bytes_mask(uint32_t nb) {  // nb in [0,8]
  return nb >= 8 ? ~0ULL : ((1ULL << (8 * nb)) - 1);
}

// kec256 of len bytes at p.  ALIGNED = true: p is 8-byte aligned and the whole
// last word is readable (arena messages); otherwise any alignment, no over-read.
template <bool ALIGNED>
KH_HD void kec256_msg(const uint8_t* p, uint32_t len, uint64_t out[4]) {
  KState s = {};
  uint32_t nfull = len / 136;
  for (uint32_t b = 0; b < nfull; ++b) {
#pragma unroll
    for (int i = 0; i < 17; ++i) kxor(s, i, ALIGNED ? ((const uint64_t*)p)[i] : load64u_n(p + 8 * i, 8));
    keccakf(s);
    p += 136;
  }
  uint32_t rem = len - nfull * 136;  // [0, 135]
#pragma unroll
  for (int i = 0; i < 17; ++i) {
    uint64_t w = 0;
    uint32_t base = 8u * (uint32_t)i;
    if (base < rem) {
      uint32_t nb = rem - base < 8 ? rem - base : 8;
      w = ALIGNED ? ((const uint64_t*)p)[i] : load64u_n(p + base, nb);
      w &= low_bytes_mask(nb);
    }
    if ((rem >> 3) == (uint32_t)i) w ^= 0x01ULL << (8 * (rem & 7));
    if (i == 16) w ^= 0x80ULL << 56;
    kxor(s, i, w);
  }
  keccakf(s);
  out[0] = lane(s, 0);
  out[1] = lane(s, 1);
  out[2] = lane(s, 2);
  out[3] = lane(s, 3);
}

// kec256 of a message shorter than one block (len <= 135) at any alignment: one
// permutation, no block loop (fewer live registers than kec256_msg's general form)
KH_HD void kec256_short(const uint8_t* p, uint32_t len, uint64_t out[4]) {
  KState s = {};
#pragma unroll
  for (int i = 0; i < 17; ++i) {
    uint64_t w = 0;
    const uint32_t base = 8u * (uint32_t)i;
    if (base < len) {
      const uint32_t nb = len - base < 8 ? len - base : 8;
      w = load64u_n(p + base, nb) & low_bytes_mask(nb);
    }
    if ((len >> 3) == (uint32_t)i) w ^= 0x01ULL << (8 * (len & 7));
    if (i == 16) w ^= 0x80ULL << 56;
    s.lo[i] = (uint32_t)w;
    s.hi[i] = (uint32_t)(w >> 32);
  }
  keccakf(s);
  out[0] = lane(s, 0);
  out[1] = lane(s, 1);
  out[2] = lane(s, 2);
  out[3] = lane(s, 3);
}

KH_HD uint32_t perms_for_len(uint32_t len) { return len / 136 + 1; }

}  // namespace khst
