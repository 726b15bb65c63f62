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


def commit_scenarios(seed=21):
    """Resident-trie commit sequences: (name, init_keys, init_vals, batches),
    batch = (upserts [(key, value)], deletes [key]).  The expected root after each batch
    is the oracle trie after put(upserts...) then remove(deletes...) in order."""
    r = random.Random(seed)
    out = []

    def acct():
        return account_value(r)

    # accounts: updates, inserts, deletes (incl. absent keys), mixed, delete + re-insert
    ks = [_rk(r) for _ in range(2000)]
    vs = [acct() for _ in ks]
    live = list(ks)
    b = []
    b.append(([(k, acct()) for k in r.sample(live, 50)], []))
    new = [_rk(r) for _ in range(30)]
    b.append(([(k, acct()) for k in new], []))
    live += new
    gone = r.sample(live, 30)
    b.append(([], gone + [_rk(r) for _ in range(5)]))
    live = [k for k in live if k not in set(gone)]
    mix_up = [(k, acct()) for k in r.sample(live, 40)] + [(_rk(r), acct()) for _ in range(40)]
    mix_del = r.sample(live, 20)
    b.append((mix_up, mix_del))
    b.append(([(gone[0], acct()), (gone[1], acct())], []))  # re-insert deleted keys
    b.append(([(live[5], vs[0])], []))                      # one update
    out.append(("accounts", ks, vs, b))

    # storage tries: 1-byte values -> inline leaves / inline branches; deletes collapse
    ks = [_rk(r) for _ in range(300)]
    vs = [storage_value(r) for _ in ks]
    b = [([(k, storage_value(r)) for k in r.sample(ks, 20)], r.sample(ks, 40)),
         ([(_rk(r), b"\x01") for _ in range(30)], []),
         ([], r.sample(ks, 100))]
    out.append(("storage", ks, vs, b))

    # deep keys: long shared prefixes (extensions), deletes that merge extensions
    ks = deep_keys(r, 120)
    vs = [codec.storage_value_rlp(i + 1) for i in range(len(ks))]
    b = [([], ks[:60:2]), ([(k, b"\x05") for k in deep_keys(r, 10, base=ks[0])], ks[1:20:3]),
         ([], ks[60:110])]
    out.append(("deep", ks, vs, b))

    # to empty and back; from empty; single key
    ks = [_rk(r) for _ in range(40)]
    vs = [acct() for _ in ks]
    out.append(("to_empty", ks, vs, [([], ks[:20]), ([], ks[20:]), ([(ks[3], acct())], []), ([(k, acct()) for k in ks[:10]], [])]))
    out.append(("from_empty", [], [], [([(k, acct()) for k in ks[:1]], []), ([(k, acct()) for k in ks[1:2]], []),
                                       ([(k, acct()) for k in ks[2:30]], []), ([], ks[:29])]))
    k1, k2 = _rk(r), _rk(r)
    out.append(("single", [k1], [acct()], [([(k1, acct())], []), ([(k2, acct())], []), ([], [k1]), ([], [k2])]))
    # the same key twice in one batch: later upsert wins; upsert + delete -> deleted
    ks = [_rk(r) for _ in range(100)]
    vs = [acct() for _ in ks]
    out.append(("same_key_batch", ks, vs, [([(ks[0], acct()), (ks[0], acct())], []), ([(ks[1], acct())], [ks[1]]),
                                          ([(ks[1], acct()), (ks[2], acct())], [ks[2], ks[2]])]))
    # a large batch relative to the trie
    ks = [_rk(r) for _ in range(2000)]
    vs = [acct() for _ in ks]
    out.append(("large_batch", ks, vs, [([(k, acct()) for k in r.sample(ks, 700)] + [(_rk(r), acct()) for _ in range(300)],
                                         r.sample(ks, 500))]))
    return out


def oracle_commits(oracle, init_keys, init_vals, batches):
    """Expected roots: the oracle trie folded put-by-put, remove-by-remove."""
    t = oracle.Trie()
    for k, v in zip(init_keys, init_vals):
        t.put(k, v)
    roots = [t.root_hash()]
    for ups, dels in batches:
        for k, v in ups:
            t.put(k, v)
        for k in dels:
            t.remove(k)
        roots.append(t.root_hash())
    return roots


def sync_node_sets(oracle, seed=31):
    """Trie nodes as a fast-sync peer returns them: (name, kind,
    {hash: encoding}) for a state trie with contract accounts and for storage tries
    whose nodes embed inline (< 32 B) children."""
    r = random.Random(seed)
    out = []
    t = oracle.Trie()
    for i in range(300):
        k = _rk(r)
        if i % 3 == 0:  # contract: non-empty storage root and code hash
            v = codec.account_rlp(r.randrange(100), r.randrange(10 ** 20), state_root=_rk(r), code_hash=_rk(r))
        elif i % 7 == 0:
            v = codec.account_rlp(0, 1, code_hash=_rk(r))
        else:
            v = account_value(r)
        t.put(k, v)
    out.append(("state", 0, t.reachable()))
    for name, keys in (("storage_deep", deep_keys(r, 120)), ("storage", [_rk(r) for _ in range(200)])):
        t = oracle.Trie()
        for i, k in enumerate(keys):
            t.put(k, codec.storage_value_rlp(r.choice([1, 5, 0x7f, 0x80, i + 1, r.randrange(1, 2 ** 64)])))
        out.append((name, 2, t.reachable()))
    return out


def mutate(r, b):
    """One random byte-level corruption of an encoding (truncate, flip, insert, delete)."""
    b = bytearray(b)
    op = r.randrange(5)
    if op == 0 and len(b) > 1:
        del b[r.randrange(1, len(b)):]
    elif op == 1 and b:
        b[r.randrange(len(b))] ^= 1 << r.randrange(8)
    elif op == 2:
        b.insert(r.randrange(len(b) + 1), r.randrange(256))
    elif op == 3 and len(b) > 1:
        del b[r.randrange(len(b))]
    elif b:
        b[r.randrange(min(len(b), 4))] = r.randrange(256)  # header bytes
    return bytes(b)


def list_key(i):
    """MptListValidator.intByteArraySerializable.toBytes: rlp.encode(i: Int)
    (MptListValidator.scala:15-18, RLPImplicits.scala:40-41, RLP.scala:238-276): 0 -> 0x80."""
    return codec.storage_value_rlp(i)


def list_cases(seed=41):
    """List tries (transactions / receipts roots): keys rlp(0..n-1) of
    1-3 bytes (the 127/128 and 255/256 index boundaries), item bytes from 1 to 300 B so
    short items give inline leaves."""
    r = random.Random(seed)
    out = []
    for n in [1, 2, 3, 16, 17, 127, 128, 129, 200, 256, 257, 1000]:
        vals = [bytes(r.getrandbits(8) for _ in range(r.choice([1, 2, 20, 60, 110, 200, 300]))) for _ in range(n)]
        out.append((f"list{n}", [list_key(i) for i in range(n)], vals))
    return out


def prefix_key_cases(seed=43):
    """Arbitrary-length keys where one key is a prefix of another: the shorter key's value
    sits in the branch's 17th slot (Node.scala:31-40, MerklePatriciaTrie.scala:207-214,263-267)."""
    r = random.Random(seed)
    out = []
    base = bytes(r.getrandbits(8) for _ in range(6))
    ks = [base[:2], base[:4], base[:4] + b"\x01", base[:4] + b"\x10", base, base[:3], b"\x00", b"\xff\xfe", b""]
    out.append(("prefix_small", ks, [bytes([i + 1]) * (i * 9 + 1) for i in range(len(ks))]))
    ks = []
    for _ in range(300):
        L = r.choice([1, 2, 3, 4, 8])
        ks.append(base[:r.randrange(0, 3)] + bytes(r.getrandbits(8) & 0x11 for _ in range(L)))
    ks = [k for k in dict.fromkeys(ks) if k]
    out.append(("prefix_random", ks, [storage_value(r) for _ in ks]))
    return out
