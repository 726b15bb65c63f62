"""GPU: the streamed host-input path of the drop-in entry points (csrc/khst.hip HostStage /
stage_host_async: keys in parts of max(n/64, 65,536) through a ring of four pinned 64-MB
chunks, each part's hashing launched as it lands; the value offsets rebased on the device;
the values last, the leaves launched behind them).  The call GenesisDataLoader.scala:139-147 /
TrieAccounts.scala:22-28 make through the JNI shim.

Every root is checked against the independent CPU batch builder (oracle/batch_root.cc, itself
pinned to the oracle and the reference's genesis fixture by tests/test_batch_root.py) and against
the device path's build of the same inputs from device buffers (no staging).  Edge cases: a key
part of one key, offsets that do not start at 0 (a caller's slice of a larger value buffer, at an
odd byte), values past one ring chunk, empty and 1-byte values, repeated keys in different
parts (the later put wins), hashed 20-byte keys, and the write-back / open entry points on the
same staging (kh_trie_root_nodes, kh_trie_open_host)."""
import ctypes

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _values(rng, n, lo, hi, empty_every=0):
    lens = rng.integers(lo, hi + 1, n)
    if empty_every:
        lens[::empty_every] = 0
    off = np.zeros(n + 1, np.uint64)
    off[1:] = np.cumsum(lens)
    return rng.integers(0, 256, int(off[-1]), dtype=np.uint8), off


def _device_root(keys, klen, vb, vo, hash_keys):
    import torch
    from khipu_amd.device import Ctx
    ctx = Ctx(0)
    n = len(vo) - 1
    dk = torch.from_numpy(np.ascontiguousarray(keys).reshape(-1)).cuda()
    dv = torch.from_numpy(np.concatenate([vb, np.zeros(64, np.uint8)])).cuda()
    do = torch.from_numpy(vo.astype(np.int64)).cuda()
    hh, _, _, _ = ctx.build(dk, klen, dv, do, n, hash_keys=hash_keys)
    return hh[0].tobytes()


CASES = [
    # name, n, klen, hash_keys, value lengths, base offset of the caller's value slice, repeats
    ("one_key_last_part", 65_537, 20, True, (60, 110), 0, 0),
    ("offset_slice_odd", 300_001, 32, False, (0, 40), 12_345, 0),
    ("values_past_a_chunk", 700_000, 32, False, (90, 110), 3, 0),
    ("repeats_across_parts", 400_000, 32, False, (1, 34), 8, 150_000),
]


@pytest.mark.parametrize("name,n,klen,hk,vlen,base,rep", CASES, ids=[c[0] for c in CASES])
def test_trie_root_host_staging(khst, oracle, name, n, klen, hk, vlen, base, rep):
    rng = np.random.default_rng(n)
    keys = rng.integers(0, 256, (n, klen), dtype=np.uint8)
    if rep:  # keys of the first parts put again in the last ones, with other values
        keys[n - rep:] = keys[:rep]
    vb, vo = _values(rng, n, *vlen, empty_every=97 if vlen[0] == 0 else 0)
    want = oracle.batch_roots(keys.reshape(-1), (vb, vo), klen=klen, hash_keys=hk, nthreads=16)[0][0]
    assert _device_root(keys, klen, vb, vo, hk) == want, name
    # the caller's values as a slice of a larger buffer: offsets start at `base`
    big = np.concatenate([rng.integers(0, 256, base, dtype=np.uint8), vb])
    st = khst.KhStats()
    got = khst.trie_root(keys.reshape(-1), (big, vo + np.uint64(base)), hash_keys=hk, klen=klen, stats=st)
    assert got == want, name
    assert st.n_inputs == n


def test_root_nodes_and_open_host_staging(khst, oracle):
    """kh_trie_root_nodes and kh_trie_open_host over the same staging (several key parts,
    offsets from a nonzero base): the root, the node set against the oracle's reachable set,
    and the opened handle's root and size."""
    from khipu_amd._lib import check, lib
    rng = np.random.default_rng(5)
    n = 140_000
    keys = [bytes(k) for k in rng.integers(0, 256, (n, 32), dtype=np.uint8)]
    vals = [bytes(rng.integers(0, 256, int(rng.integers(1, 60)), dtype=np.uint8)) for _ in range(n)]
    want = oracle.batch_root(keys, vals, nthreads=16)
    root, nodes = khst.trie_root_nodes(keys, vals)
    assert root == want
    o = oracle.Trie()
    for k, v in zip(keys[:20_000], vals[:20_000]):  # (the oracle's node set on a prefix: size of the check)
        o.put(k, v)
    r2, n2 = khst.trie_root_nodes(keys[:20_000], vals[:20_000])
    assert r2 == o.root_hash() and n2 == o.reachable()
    assert all(khst.kec256(e) == h for h, e in nodes.items() if len(e) >= 32)
    kb = np.frombuffer(b"".join(keys), np.uint8)
    blob = b"".join(vals)
    base = 77
    vb = np.frombuffer(bytes(base) + blob, np.uint8)
    vo = np.zeros(n + 1, np.uint64)
    vo[1:] = np.cumsum([len(v) for v in vals])
    vo += np.uint64(base)
    h = ctypes.c_void_p()
    out = np.zeros(32, np.uint8)
    check(lib().kh_trie_open_host(kb.ctypes.data, 32, vb.ctypes.data, vo.ctypes.data, n, 0, out.ctypes.data,
                                  ctypes.byref(h)))
    try:
        assert out.tobytes() == want
    finally:
        lib().kh_trie_free(h)
