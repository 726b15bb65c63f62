"""The independent CPU batch builder (oracle/batch_root.cc, test infrastructure) against
the khipu-faithful sequential oracle (oracle/khipu_oracle.cc) — so that it can check the
GPU roots at sizes the sequential oracle cannot reach (100M accounts in bench.py)."""
import random

import numpy as np
import pytest

from tests import cases as C

GENESIS_ROOT = "d7f8974fb5ac78d9ac099b9ad5018bedc2ce0a72dad1827a1709da30580f0544"


def test_batch_keccak_vs_oracle(oracle):
    r = random.Random(1)
    for L in list(range(0, 300)) + [407, 408, 409, 543, 544, 545, 1000]:
        m = bytes(r.getrandbits(8) for _ in range(L))
        assert oracle.batch_kec256(m) == oracle.kec256(m), L


@pytest.mark.parametrize("case", C.all_cases(), ids=lambda c: c[0])
def test_batch_root_vs_seq(oracle, case):
    name, keys, vals = case
    assert oracle.batch_root(keys, vals, klen=32, nthreads=3) == oracle.seq_root(keys, vals), name


def test_batch_segmented_vs_seq(oracle):
    tries = C.segmented_case()
    keys = [k for ks, _ in tries for k in ks]
    vals = [v for _, vs in tries for v in vs]
    so = np.cumsum([0] + [len(ks) for ks, _ in tries])
    roots, st = oracle.batch_roots(keys, vals, klen=32, seg_off=so, nthreads=4)
    for (ks, vs), g in zip(tries, roots):
        assert g == (oracle.seq_root(ks, vs) if ks else oracle.kec256(b"\x80"))


@pytest.mark.parametrize("case", C.list_cases() + C.prefix_key_cases(), ids=lambda c: c[0])
def test_batch_variable_keys_vs_seq(oracle, case):
    """List tries (rlp(i) keys, MptListValidator.scala:30-46) and keys that are prefixes of
    other keys (branch values): the sequential oracle handles any key length."""
    name, keys, vals = case
    t = oracle.Trie()
    for k, v in zip(keys, vals):
        t.put(k, v)
    assert oracle.batch_root(keys, vals, nthreads=2) == t.root_hash(), name


def test_batch_genesis(oracle):
    import __graft_entry__ as g
    addrs, vals = g._genesis_inputs()
    roots, st = oracle.batch_roots(addrs, vals, klen=20, hash_keys=True, nthreads=4)
    assert roots[0].hex() == GENESIS_ROOT
    assert st["leaves"] == st["distinct"] == 8893 and st["key_perms"] == 8893


def test_batch_random_accounts_parallel_spine(oracle):
    """100k random accounts: the threaded spine/subtree split (m >= 20000) against the
    sequential fold, and thread-count invariance."""
    r = np.random.default_rng(5)
    n = 100_000
    keys = r.integers(0, 256, n * 32, dtype=np.uint8)
    lens = r.integers(70, 80, n)
    voff = np.zeros(n + 1, np.uint64)
    voff[1:] = np.cumsum(lens)
    vb = r.integers(0, 256, int(voff[-1]) + 8, dtype=np.uint8)
    exp = oracle.seq_root_packed(keys, 32, vb, voff, n)
    for nt in (1, 5, 16):
        roots, st = oracle.batch_roots(keys, (vb, voff), klen=32, nthreads=nt)
        assert roots[0] == exp, nt
    assert st["leaves"] == n and st["node_hashes"] > n
