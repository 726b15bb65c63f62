"""Seeded input sets shared by the CPU (host replay) and GPU parity tests.

Each case is (name, keys32, values); the expected root comes from the oracle
(oracle/khipu_oracle.cc, the khipu-faithful sequential MerklePatriciaTrie).
Edge cases follow SURVEY.md Appendix A and §8(c): inline (< 32 B) nodes from
1-byte storage values, keys sharing 63 nibbles, an extension at the root,
duplicate keys (later put wins), values around the RLP 55/56 and 255/256
length thresholds, empty values, and keys tying on their first 8 bytes (the
full-key sort path).
"""
import random

from khipu_amd import codec


def _rk(r):
    return bytes(r.getrandbits(8) for _ in range(32))


def storage_value(r):
    return codec.storage_value_rlp(r.choice([1, 0x7F, 0x80, 0xFF, r.randrange(1, 2 ** 256), r.randrange(1, 2 ** 40)]))


def account_value(r, i=None):
    return codec.account_rlp(r.randrange(1 << 16) if i is None else i, r.randrange(10 ** 22))


def deep_keys(r, n, base=None):
    base = bytearray(base or _rk(r))
    out = []
    for _ in range(n):
        b = bytearray(base)
        b[31] = r.randrange(256)
        b[30] ^= r.randrange(4)
        b[29] ^= r.randrange(2)
        out.append(bytes(b))
    return list(dict.fromkeys(out))


def all_cases(seed=11, big=True):
    r = random.Random(seed)
    cases = []
    for n in [1, 2, 3, 16, 17, 100, 1000] + ([10000] if big else []):
        ks = [_rk(r) for _ in range(n)]
        cases.append((f"accounts{n}", ks, [account_value(r) for _ in ks]))
    for n in [2, 5, 30, 300, 3000]:
        ks = [_rk(r) for _ in range(n)]
        cases.append((f"storage{n}", ks, [storage_value(r) for _ in ks]))
    for n in [2, 3, 16, 40, 200]:
        ks = deep_keys(r, n)
        cases.append((f"deep_acct{n}", ks, [codec.account_rlp(i, 2) for i in range(len(ks))]))
        cases.append((f"deep_stor{n}", ks, [codec.storage_value_rlp(i + 1) for i in range(len(ks))]))
    b0 = bytearray(_rk(r))
    b1 = bytearray(b0)
    b1[31] ^= 0x01
    cases.append(("shared63", [bytes(b0), bytes(b1)], [b"\x01", b"\x02"]))
    b2 = bytearray(b0)
    b2[31] ^= 0x10
    cases.append(("shared62", [bytes(b0), bytes(b2)], [b"\x05", codec.account_rlp(1, 1)]))
    ks = []
    for _ in range(50):
        b = bytearray(_rk(r))
        b[0] = 0xAB
        b[1] = (b[1] & 0x0F) | 0xC0
        ks.append(bytes(b))
    cases.append(("root_ext", ks, [storage_value(r) for _ in ks]))
    ks = [_rk(r) for _ in range(20)]
    ks2 = ks + [ks[3], ks[7], ks[3], ks[0]]
    cases.append(("duplicates", ks2, [storage_value(r) for _ in ks2]))
    ks = [_rk(r) for _ in range(40)]
    cases.append(("long_values", ks, [bytes(r.getrandbits(8) for _ in range(r.choice([1, 2, 55, 56, 60, 200, 255, 256,
                                                                                           300, 1000])))
                                      for _ in ks]))
    cases.append(("empty_values", ks[:5], [b""] * 5))
    # first 8 bytes equal -> a run of 64 equal sort prefixes, fixed locally (k_tie_fix)
    pre = _rk(r)[:8]
    ks = [pre + _rk(r)[8:] for _ in range(64)] + [_rk(r) for _ in range(64)]
    cases.append(("prefix_ties", ks, [account_value(r) for _ in ks]))
    ks = [pre + _rk(r)[8:] for _ in range(10)]
    ks = ks + ks[:4]
    cases.append(("prefix_ties_dups", ks, [storage_value(r) for _ in ks]))
    # a run longer than TIE_RUN_MAX (64) -> the full 256-bit sort path
    ks = [pre[:4] + _rk(r)[4:] for _ in range(150)] + [_rk(r) for _ in range(30)]
    ks = ks + ks[5:9]
    cases.append(("prefix_ties_long", ks, [storage_value(r) for _ in ks]))
    return cases


def segmented_case(seed=5, nseg=40):
    r = random.Random(seed)
    tries = []
    for s in range(nseg):
        k = r.choice([0, 1, 2, 3, 17, 60, 200])
        ks = [_rk(r) for _ in range(k)]
        if s % 7 == 3 and k > 4:
            ks[1] = ks[0]  # duplicate inside one trie
        tries.append((ks, [storage_value(r) for _ in ks]))
    # identical key in two different tries must not merge
    if tries[5][0] and tries[6][0]:
        tries[6][0][0] = tries[5][0][0]
    return tries
