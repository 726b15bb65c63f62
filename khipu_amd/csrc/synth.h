// Deterministic synthetic accounts, counter-based so any slice can be
// regenerated on any device or on the host.  Account i of config cfg:
//   draw(j)  = splitmix64 output j of seed 0x6b68697075000000 | cfg
//   d_q      = draw(8i + q)
//   address  = LE(d0) || LE(d1) || LE(d2)[0..4)                  (20 B)
//   nonce    = d3 >> 63 ? 0 : d3 & 0xFFFF
//   balance  = big-endian value of the first ((d3 >> 16) % 13) bytes of LE(d4) || LE(d5)
//   contract = ((d3 >> 32) % 10) == 0:
//              stateRoot = kec256(LE64(i)), codeHash = kec256(LE64(~i))
//              else EMPTY_TRIE_HASH / EMPTY_CODE_HASH (domain/Account.scala:13-17)
//   body     = RLP[nonce, balance, stateRoot, codeHash]          (PV63.scala:46-51)
// with integers as minimal big-endian strings, zero as "" (rlp/package.scala:56-57).
#pragma once
#include <math.h>

#include "trie_ops.h"

namespace khst {

KH_HD uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
  return z ^ (z >> 31);
}
KH_HD uint64_t synth_draw(uint32_t cfg, uint64_t j) {
  uint64_t seed = 0x6b68697075000000ULL | cfg;
  return mix64(seed + (j + 1) * 0x9E3779B97F4A7C15ULL);
}

struct SynthAcct {
  uint64_t addr[3];  // 20 bytes LE
  uint64_t nonce;
  uint32_t blen;      // minimal balance length
  uint64_t bal_hi, bal_lo;  // balance value (up to 96 bits): hi = top 32 bits
  bool contract;
};

KH_HD SynthAcct synth_acct(uint32_t cfg, uint64_t i) {
  uint64_t d[6];
  for (int q = 0; q < 6; ++q) d[q] = synth_draw(cfg, 8 * i + q);
  SynthAcct a;
  a.addr[0] = d[0];
  a.addr[1] = d[1];
  a.addr[2] = d[2] & 0xFFFFFFFFULL;
  a.nonce = (d[3] >> 63) ? 0 : (d[3] & 0xFFFF);
  uint32_t bl = (uint32_t)((d[3] >> 16) % 13);
  // value = big-endian of bytes b[0..bl) where b = LE(d4) || LE(d5)
  uint64_t hi = 0, lo = 0;  // 128-bit accumulator (only 96 bits used)
  for (uint32_t q = 0; q < bl; ++q) {
    uint32_t byte = q < 8 ? (uint32_t)(d[4] >> (8 * q)) & 0xFF : (uint32_t)(d[5] >> (8 * (q - 8))) & 0xFF;
    hi = (hi << 8) | (lo >> 56);
    lo = (lo << 8) | byte;
  }
  a.bal_hi = hi;
  a.bal_lo = lo;
  uint32_t n = 0;
  if (hi)
    n = 8 + be_nbytes(hi);
  else
    n = be_nbytes(lo);
  a.blen = n;
  a.contract = ((d[3] >> 32) % 10) == 0;
  return a;
}

KH_HD uint32_t synth_uint_str_len(uint32_t nb, uint32_t first) {
  return (uint32_t)rlp_str_len(nb, first);
}

KH_HD uint32_t synth_body_payload(const SynthAcct& a) {
  uint32_t nn = be_nbytes(a.nonce);
  uint32_t nfirst = nn ? (uint32_t)(a.nonce >> (8 * (nn - 1))) & 0xFF : 0;
  uint32_t bfirst = 0;
  if (a.blen > 8)
    bfirst = (uint32_t)(a.bal_hi >> (8 * (a.blen - 9))) & 0xFF;
  else if (a.blen)
    bfirst = (uint32_t)(a.bal_lo >> (8 * (a.blen - 1))) & 0xFF;
  return synth_uint_str_len(nn, nfirst) + synth_uint_str_len(a.blen, bfirst) + 33 + 33;
}
KH_HD uint32_t synth_body_len(const SynthAcct& a) {
  uint32_t payload = synth_body_payload(a);
  return rlp_hdr_len(payload) + payload;
}

// Writes the body at dst (any alignment) byte by byte; returns its length.
KH_HD uint32_t synth_body_write(const SynthAcct& a, uint64_t i, uint8_t* dst) {
  uint8_t buf[96];
  uint32_t n = 0;
  uint32_t nn = be_nbytes(a.nonce);
  uint32_t payload = synth_body_payload(a);  // 68..82 bytes
  if (payload < 56) {
    buf[n++] = (uint8_t)(0xC0 + payload);
  } else {
    buf[n++] = 0xF8;
    buf[n++] = (uint8_t)payload;
  }
  // nonce
  if (nn == 0) {
    buf[n++] = 0x80;
  } else {
    uint32_t first = (uint32_t)(a.nonce >> (8 * (nn - 1))) & 0xFF;
    if (!(nn == 1 && first < 0x80)) buf[n++] = (uint8_t)(0x80 + nn);
    for (int q = (int)nn - 1; q >= 0; --q) buf[n++] = (uint8_t)(a.nonce >> (8 * q));
  }
  // balance
  if (a.blen == 0) {
    buf[n++] = 0x80;
  } else {
    uint8_t bb[12];
    for (uint32_t q = 0; q < a.blen; ++q) {
      uint32_t pos = a.blen - 1 - q;  // byte index from the least significant end
      bb[q] = pos >= 8 ? (uint8_t)(a.bal_hi >> (8 * (pos - 8))) : (uint8_t)(a.bal_lo >> (8 * pos));
    }
    if (!(a.blen == 1 && bb[0] < 0x80)) buf[n++] = (uint8_t)(0x80 + a.blen);
    for (uint32_t q = 0; q < a.blen; ++q) buf[n++] = bb[q];
  }
  uint64_t sr[4], ch[4];
  if (a.contract) {
    uint64_t m1[2] = {i, 0}, m2[2] = {~i, 0};
    kec256_msg<true>((const uint8_t*)m1, 8, sr);
    kec256_msg<true>((const uint8_t*)m2, 8, ch);
  } else {
    // EMPTY_TRIE_HASH 56e81f17...b421 and EMPTY_CODE_HASH c5d24601...a470 as LE words
    sr[0] = 0xa655cc1b171fe856ULL; sr[1] = 0x6ef8c092e64583ffULL; sr[2] = 0xc0ad6c991be0485bULL;
    sr[3] = 0x21b463e3b52f6201ULL;
    ch[0] = 0x3c23f7860146d2c5ULL; ch[1] = 0xc003c7dcb27d7e92ULL; ch[2] = 0x3b2782ca53b600e5ULL;
    ch[3] = 0x70a4855d04d8fa7bULL;
  }
  buf[n++] = 0xA0;
  for (int q = 0; q < 32; ++q) buf[n++] = (uint8_t)(sr[q >> 3] >> (8 * (q & 7)));
  buf[n++] = 0xA0;
  for (int q = 0; q < 32; ++q) buf[n++] = (uint8_t)(ch[q >> 3] >> (8 * (q & 7)));
  for (uint32_t q = 0; q < n; ++q) dst[q] = buf[q];
  return n;
}

KH_HD void synth_addr_write(const SynthAcct& a, uint8_t* dst) {
  for (int q = 0; q < 20; ++q) dst[q] = (uint8_t)(a.addr[q >> 3] >> (8 * (q & 7)));
}

// Synthetic contract storage tries (BASELINE configs[3]), counter-based
// per trie so any range of tries can be generated on any GPU:
//   slots(t) = clamp(floor(exp(u * ln(10^4 + 1))), 1, 10^4), u = draw(t) / 2^64
//              (log-uniform in [1, 10^4]; mean ~1.1k slots)
//   slot i   : key = the 32-byte big-endian i (DataWord; hashed with KH_HASH_KEYS as
//              hashDataWordSerializable does, trie/package.scala:34-36)
//              value = RLP(b[0..L)) with w_q = draw(4 * (2^40 + 16384 t + i) + q),
//              L = 1 + (w_3 >> 56) % 32, b = LE(w_0..w_3), b[0] forced non-zero (a trimmed
//              DataWord, rlpDataWordSerializer, trie/package.scala:28-32): a 1-byte value
//              < 0x80 is its own encoding (inline leaves occur)
// The device's exp is the only floating-point step: every GPU generates the same data, and
// CPU checks read the generated buffers back.
constexpr uint32_t SYNTH_STORAGE_MAX_SLOTS = 10000;
KH_HD uint32_t synth_storage_slots(uint32_t cfg, uint64_t t) {
  const double u = (double)(synth_draw(cfg, t) >> 11) * (1.0 / 9007199254740992.0);
  double c = exp(u * log((double)SYNTH_STORAGE_MAX_SLOTS + 1.0));
  if (c < 1.0) c = 1.0;
  if (c > (double)SYNTH_STORAGE_MAX_SLOTS) c = (double)SYNTH_STORAGE_MAX_SLOTS;
  return (uint32_t)c;
}
struct SynthSlot {
  uint64_t w[4];
  uint32_t L;    // value bytes
  uint32_t enc;  // RLP-encoded length
};
KH_HD SynthSlot synth_slot(uint32_t cfg, uint64_t t, uint32_t i) {
  SynthSlot s;
  const uint64_t j = 4 * ((1ULL << 40) + 16384ULL * t + i);
  for (int q = 0; q < 4; ++q) s.w[q] = synth_draw(cfg, j + q);
  if ((s.w[0] & 0xFF) == 0) s.w[0] |= 1;
  s.L = 1 + (uint32_t)((s.w[3] >> 56) % 32);
  s.enc = (s.L == 1 && (s.w[0] & 0xFF) < 0x80) ? 1 : s.L + 1;
  return s;
}
KH_HD void synth_slot_write(const SynthSlot& s, uint32_t i, uint8_t* key32, uint8_t* val) {
  for (int q = 0; q < 32; ++q) key32[q] = q < 28 ? 0 : (uint8_t)(i >> (8 * (31 - q)));
  uint32_t n = 0;
  if (s.enc != 1) val[n++] = (uint8_t)(0x80 + s.L);
  for (uint32_t q = 0; q < s.L; ++q) val[n++] = (uint8_t)(s.w[q >> 3] >> (8 * (q & 7)));
}

}  // namespace khst
