"""List tries and variable-length keys on the GPU against the oracle.

Transactions / receipts roots put item i under rlp(i) (MptListValidator.scala:15-46,
BlockGenerator.scala:157-163): 1-3 byte keys, so the trie has branches at depth 0/1 and
short keys.  Generic unhashed keys of other lengths may prefix each other; the shorter
key's value then sits in the branch's 17th slot (Node.scala:31-40).  Both go through
kh_list_roots / kh_trie_roots_varkeys; the checker is the sequential oracle
(oracle/khipu_oracle.cc, khipu's put/fix restated) and the batch builder."""
import random

import pytest

from tests import cases as C

pytestmark = pytest.mark.gpu

EMPTY = bytes.fromhex("56e81f171bcc55a6ff8345e692c0f86e5b48e01b996cadc001622fb5e363b421")


def _seq_root(oracle, keys, vals):
    t = oracle.Trie()
    for k, v in zip(keys, vals):
        t.put(k, v)
    return t.root_hash()


@pytest.mark.parametrize("case", C.list_cases(), ids=lambda c: c[0])
def test_list_roots_vs_oracle(oracle, case):
    from khipu_amd.trie import list_roots, trie_roots_varkeys, MptListValidator
    name, keys, vals = case
    exp = _seq_root(oracle, keys, vals)
    assert list_roots([vals])[0] == exp, name          # keys rlp(i) made on the device
    assert trie_roots_varkeys([(keys, vals)])[0] == exp, name  # the same keys given by the caller
    assert MptListValidator.is_valid(exp, vals)


def test_list_roots_many_blocks(oracle):
    """One call for many blocks' lists (segments), including empty lists and 0..1000 items."""
    from khipu_amd.trie import list_roots
    r = random.Random(7)
    lists = []
    for n in [0, 1, 0, 5, 127, 128, 129, 300, 1000, 2, 0, 33]:
        lists.append([bytes(r.getrandbits(8) for _ in range(r.choice([1, 3, 31, 32, 33, 90, 140, 400])))
                      for _ in range(n)])
    got = list_roots(lists)
    for it, g in zip(lists, got):
        exp = _seq_root(oracle, [C.list_key(i) for i in range(len(it))], it) if it else EMPTY
        assert g == exp, len(it)


@pytest.mark.parametrize("case", C.prefix_key_cases(), ids=lambda c: c[0])
def test_prefix_keys_vs_oracle(oracle, case):
    from khipu_amd.trie import trie_roots_varkeys
    name, keys, vals = case
    exp = _seq_root(oracle, keys, vals)
    assert trie_roots_varkeys([(keys, vals)])[0] == exp, name
    assert oracle.batch_root(keys, vals, nthreads=2) == exp, name


def test_varkeys_edge_cases(oracle):
    """Empty key (the root branch's value), a lone empty key, duplicate puts (later wins),
    one-byte values < 0x80 (raw RLP), long branch values (> one Keccak block), 32-byte keys
    mixed with shorter ones, and segments."""
    from khipu_amd.trie import trie_roots_varkeys
    r = random.Random(11)
    big = bytes(r.getrandbits(8) for _ in range(300))
    tries = [
        ([b"", b"\x01"], [b"\x05", b"abc"]),
        ([b""], [b"zz"]),
        ([b"\x12\x34", b"\x12", b"\x12\x34"], [b"a", b"\x7f", b"c" * 40]),
        ([b"\xab", b"\xab\xcd", b"\xab\xce"], [big, b"\x01", b"\x02"]),
        ([bytes(32), bytes(31), bytes(1), b""], [b"1", b"2" * 50, b"3", b"\x80"]),
        ([bytes([i]) * (1 + i % 7) for i in range(60)], [bytes([i]) * (1 + i % 45) for i in range(60)]),
        ([], []),
    ]
    got = trie_roots_varkeys(tries)
    for (ks, vs), g in zip(tries, got):
        if not ks:
            assert g == EMPTY
            continue
        assert g == _seq_root(oracle, ks, vs), ks[:4]


def _last_wins(ks, vs):
    d = {}
    for k, v in zip(ks, vs):
        d[k] = v
    return list(d), list(d.values())


def test_varkeys_ties_and_full_sort(oracle):
    """More than TIE_RUN_MAX keys sharing their first 4 bytes (the full-key sort path) with
    prefix relations and repeated puts inside the run.

    Repeated puts: the engine keeps the last put of a key (the batch contract of
    TrieAccounts.flush / TrieStorage.flush, which put each key once).  The reference's fold
    over a REPEATED key whose leaf has no path left turns that leaf into a value-only
    branch (putInLeafNode, MerklePatriciaTrie.scala:187-199: ml == 0 with an empty
    existing key) -- history-dependent and never reached by its callers (one put per key
    and per list index) -- so the expected root is the fold over the last-wins puts
    ("repeated puts")."""
    from khipu_amd.trie import trie_roots_varkeys
    from khipu_amd._lib import KhStats
    r = random.Random(13)
    base = b"\x42\x42\x42\x42"
    ks = [base + bytes(r.getrandbits(8) & 0x0F for _ in range(r.randrange(0, 5))) for _ in range(400)]
    vs = [bytes([r.getrandbits(8)]) * r.choice([1, 2, 40]) for _ in ks]
    st = KhStats()
    got = trie_roots_varkeys([(ks, vs)], stats=st)[0]
    dk, dv = _last_wins(ks, vs)
    assert len(dk) < len(ks)
    assert got == _seq_root(oracle, dk, dv)
    assert got == oracle.batch_root(ks, vs, nthreads=2)
    assert st.full_sort == 1 and st.n_leaves == len(dk)
    got2 = trie_roots_varkeys([(dk, dv)], stats=st)[0]
    assert got2 == got


def test_varkeys_repeated_puts_short_runs(oracle):
    """Repeated puts of 1-2 byte keys (the tie-fix path, no full sort): last put wins."""
    from khipu_amd.trie import trie_roots_varkeys
    r = random.Random(2)
    ks = [bytes(r.getrandbits(8) for _ in range(r.randrange(1, 3))) for _ in range(300)]
    vs = [bytes([i % 256]) * 3 for i in range(len(ks))]
    dk, dv = _last_wins(ks, vs)
    assert len(dk) < len(ks)
    assert trie_roots_varkeys([(ks, vs)])[0] == _seq_root(oracle, dk, dv)


def test_varkeys_rejects_long_keys():
    from khipu_amd.trie import trie_roots_varkeys
    from khipu_amd._lib import MPTException
    with pytest.raises(MPTException):
        trie_roots_varkeys([([bytes(33)], [b"x"])])


def test_dev_list_roots_matches_host(oracle):
    """kh_dev_list_roots (items in HBM, segment ids and rlp(i) keys made on the device)
    against the host entry point and the oracle, including empty lists and a sub-range of
    the item offsets (seg_off[0] > 0)."""
    import numpy as np
    import torch
    import bench
    from khipu_amd.device import Ctx
    from khipu_amd.trie import list_roots
    items, off, so = bench.list_workload(60, seed=3)
    so[5] = so[4]  # an empty list
    so[6] = so[4]
    lists = [[items[int(off[j]):int(off[j + 1])].tobytes() for j in range(int(so[b]), int(so[b + 1]))]
             for b in range(len(so) - 1)]
    ctx = Ctx(0)
    d_items = torch.from_numpy(items).to("cuda:0")
    d_off = torch.from_numpy(off.astype(np.int64)).to("cuda:0")
    got, st = ctx.list_roots(d_items, d_off, so)
    assert got == list_roots(lists)
    for b in (0, 4, 5, 17, 59):
        exp = _seq_root(oracle, [C.list_key(i) for i in range(len(lists[b]))], lists[b]) if lists[b] else EMPTY
        assert got[b] == exp, b
    sub, _ = ctx.list_roots(d_items, d_off, so[10:21])
    assert sub == got[10:20]
