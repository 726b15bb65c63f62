// Keccak-256 (legacy 0x01 padding) for gfx950: one message per lane, the 25-lane
// Keccak-f[1600] state held in 50 VGPRs.
//
// Reference behaviour: khipu-base/.../crypto/hash/KeccakCore.scala:39-52 (RC),
// :103-531 (processBlock), :534-562 (doPadding: 0x01 .. 0x80, 0x81 if one byte
// is left), :570 (rate 136 B); DigestEngine.scala:102-166 (a block is absorbed
// as soon as 136 bytes are buffered, so L bytes cost floor(L/136)+1 permutations).
//
// gfx950 has no 64-bit logic or rotate instructions: the compiler splits each
// 64-bit op into two 32-bit halves (v_xor3_b32 for theta's 5-way XOR,
// v_alignbit_b32 pairs for rho, v_bfi_b32 + v_xor_b32 for chi).  All state
// indices are compile-time constants so the state never leaves registers.
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

KH_HD uint64_t rotl64(uint64_t x, int n) { return (x << n) | (x >> (64 - n)); }

// chi term a ^ (~b & c), written as a bit-select so it lowers to v_bfi_b32.
KH_HD uint64_t chi(uint64_t a, uint64_t b, uint64_t c) { return a ^ (~b & c); }

// One Keccak-f[1600] round on named state words (rho/pi folded into renaming).
#define KH_ROUND(rc)                                                                   \
  {                                                                                    \
    uint64_t C0 = a00 ^ a05 ^ a10 ^ a15 ^ a20, C1 = a01 ^ a06 ^ a11 ^ a16 ^ a21;       \
    uint64_t C2 = a02 ^ a07 ^ a12 ^ a17 ^ a22, C3 = a03 ^ a08 ^ a13 ^ a18 ^ a23;       \
    uint64_t C4 = a04 ^ a09 ^ a14 ^ a19 ^ a24;                                         \
    uint64_t D0 = C4 ^ rotl64(C1, 1), D1 = C0 ^ rotl64(C2, 1), D2 = C1 ^ rotl64(C3, 1); \
    uint64_t D3 = C2 ^ rotl64(C4, 1), D4 = C3 ^ rotl64(C0, 1);                         \
    uint64_t b00 = a00 ^ D0;                                                           \
    uint64_t b10 = rotl64(a01 ^ D1, 1);                                                \
    uint64_t b20 = rotl64(a02 ^ D2, 62);                                               \
    uint64_t b05 = rotl64(a03 ^ D3, 28);                                               \
    uint64_t b15 = rotl64(a04 ^ D4, 27);                                               \
    uint64_t b16 = rotl64(a05 ^ D0, 36);                                               \
    uint64_t b01 = rotl64(a06 ^ D1, 44);                                               \
    uint64_t b11 = rotl64(a07 ^ D2, 6);                                                \
    uint64_t b21 = rotl64(a08 ^ D3, 55);                                               \
    uint64_t b06 = rotl64(a09 ^ D4, 20);                                               \
    uint64_t b07 = rotl64(a10 ^ D0, 3);                                                \
    uint64_t b17 = rotl64(a11 ^ D1, 10);                                               \
    uint64_t b02 = rotl64(a12 ^ D2, 43);                                               \
    uint64_t b12 = rotl64(a13 ^ D3, 25);                                               \
    uint64_t b22 = rotl64(a14 ^ D4, 39);                                               \
    uint64_t b23 = rotl64(a15 ^ D0, 41);                                               \
    uint64_t b08 = rotl64(a16 ^ D1, 45);                                               \
    uint64_t b18 = rotl64(a17 ^ D2, 15);                                               \
    uint64_t b03 = rotl64(a18 ^ D3, 21);                                               \
    uint64_t b13 = rotl64(a19 ^ D4, 8);                                                \
    uint64_t b14 = rotl64(a20 ^ D0, 18);                                               \
    uint64_t b24 = rotl64(a21 ^ D1, 2);                                                \
    uint64_t b09 = rotl64(a22 ^ D2, 61);                                               \
    uint64_t b19 = rotl64(a23 ^ D3, 56);                                               \
    uint64_t b04 = rotl64(a24 ^ D4, 14);                                               \
    a00 = chi(b00, b01, b02) ^ (rc);                                                   \
    a01 = chi(b01, b02, b03);                                                          \
    a02 = chi(b02, b03, b04);                                                          \
    a03 = chi(b03, b04, b00);                                                          \
    a04 = chi(b04, b00, b01);                                                          \
    a05 = chi(b05, b06, b07);                                                          \
    a06 = chi(b06, b07, b08);                                                          \
    a07 = chi(b07, b08, b09);                                                          \
    a08 = chi(b08, b09, b05);                                                          \
    a09 = chi(b09, b05, b06);                                                          \
    a10 = chi(b10, b11, b12);                                                          \
    a11 = chi(b11, b12, b13);                                                          \
    a12 = chi(b12, b13, b14);                                                          \
    a13 = chi(b13, b14, b10);                                                          \
    a14 = chi(b14, b10, b11);                                                          \
    a15 = chi(b15, b16, b17);                                                          \
    a16 = chi(b16, b17, b18);                                                          \
    a17 = chi(b17, b18, b19);                                                          \
    a18 = chi(b18, b19, b15);                                                          \
    a19 = chi(b19, b15, b16);                                                          \
    a20 = chi(b20, b21, b22);                                                          \
    a21 = chi(b21, b22, b23);                                                          \
    a22 = chi(b22, b23, b24);                                                          \
    a23 = chi(b23, b24, b20);                                                          \
    a24 = chi(b24, b20, b21);                                                          \
  }

struct KState {
  uint64_t a00, a01, a02, a03, a04, a05, a06, a07, a08, a09, a10, a11, a12, a13, a14, a15, a16, a17, a18,
      a19, a20, a21, a22, a23, a24;
};

KH_HD void keccakf(KState& s) {
  uint64_t a00 = s.a00, a01 = s.a01, a02 = s.a02, a03 = s.a03, a04 = s.a04, a05 = s.a05, a06 = s.a06,
           a07 = s.a07, a08 = s.a08, a09 = s.a09, a10 = s.a10, a11 = s.a11, a12 = s.a12, a13 = s.a13,
           a14 = s.a14, a15 = s.a15, a16 = s.a16, a17 = s.a17, a18 = s.a18, a19 = s.a19, a20 = s.a20,
           a21 = s.a21, a22 = s.a22, a23 = s.a23, a24 = s.a24;
#pragma unroll 2
  for (int r = 0; r < 24; ++r) KH_ROUND(round_constant(r));
  s.a00 = a00; s.a01 = a01; s.a02 = a02; s.a03 = a03; s.a04 = a04; s.a05 = a05; s.a06 = a06;
  s.a07 = a07; s.a08 = a08; s.a09 = a09; s.a10 = a10; s.a11 = a11; s.a12 = a12; s.a13 = a13;
  s.a14 = a14; s.a15 = a15; s.a16 = a16; s.a17 = a17; s.a18 = a18; s.a19 = a19; s.a20 = a20;
  s.a21 = a21; s.a22 = a22; s.a23 = a23; s.a24 = a24;
}

// XOR word w into rate lane i (i compile-time after unrolling).
KH_HD void kxor(KState& s, int i, uint64_t w) {
  switch (i) {
    case 0: s.a00 ^= w; break;
    case 1: s.a01 ^= w; break;
    case 2: s.a02 ^= w; break;
    case 3: s.a03 ^= w; break;
    case 4: s.a04 ^= w; break;
    case 5: s.a05 ^= w; break;
    case 6: s.a06 ^= w; break;
    case 7: s.a07 ^= w; break;
    case 8: s.a08 ^= w; break;
    case 9: s.a09 ^= w; break;
    case 10: s.a10 ^= w; break;
    case 11: s.a11 ^= w; break;
    case 12: s.a12 ^= w; break;
    case 13: s.a13 ^= w; break;
    case 14: s.a14 ^= w; break;
    case 15: s.a15 ^= w; break;
    case 16: s.a16 ^= w; break;
  }
}

// nb (1..8) little-endian bytes from an arbitrary address via aligned 8-byte
// loads; only the aligned words holding bytes [p, p+nb) are read, so no access
// leaves the 8-byte-aligned span of the message.  Bytes above nb are garbage.
KH_HD uint64_t load64u_n(const uint8_t* p, uint32_t nb) {
  uintptr_t a = (uintptr_t)p;
  const uint64_t* q = (const uint64_t*)(a & ~(uintptr_t)7);
  uint32_t off = (uint32_t)(a & 7);
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
  out[0] = s.a00;
  out[1] = s.a01;
  out[2] = s.a02;
  out[3] = s.a03;
}

KH_HD uint32_t perms_for_len(uint32_t len) { return len / 136 + 1; }

}  // namespace khst
