"""BASELINE.json configs at their configured shapes on the GPU, checked against the
independent CPU batch builder (oracle/batch_root.cc) for every root and against the
khipu-faithful sequential oracle on sampled tries."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def storage_tries(rng, ntries, lo=1, hi=10_000):
    """configs[3]: ntries contract storage tries, slot counts log-uniform in [lo, hi]; slot
    key = kec256(32-byte big-endian slot index) (hashDataWordSerializable,
    trie/package.scala:34-36) -> raw 32-byte keys hashed on the device; value =
    RLP(trimmed 1-32 random bytes) (rlpDataWordSerializer, trie/package.scala:28-32), so
    1-byte values < 0x80 (inline leaves) occur."""
    cnt = np.exp(rng.uniform(np.log(lo), np.log(hi + 1), ntries)).astype(np.int64).clip(lo, hi)
    seg_off = np.zeros(ntries + 1, np.uint64)
    seg_off[1:] = np.cumsum(cnt)
    n = int(seg_off[-1])
    keys = np.zeros((n, 32), np.uint8)
    keys[:, 24:] = rng.integers(0, 1 << 20, n, dtype=np.uint64).astype(">u8").view(np.uint8).reshape(n, 8)
    vlen = rng.integers(1, 33, n)
    first = rng.integers(1, 256, n).astype(np.uint8)  # trimmed: no leading zero byte
    raw1 = (vlen == 1) & (first < 0x80)
    enc_len = np.where(raw1, 1, vlen + 1)
    voff = np.zeros(n + 1, np.uint64)
    voff[1:] = np.cumsum(enc_len)
    vb = rng.integers(0, 256, int(voff[-1]) + 8, dtype=np.uint8)
    st = voff[:-1].astype(np.int64)
    vb[st[~raw1]] = (0x80 + vlen[~raw1]).astype(np.uint8)
    vb[st[~raw1] + 1] = first[~raw1]
    vb[st[raw1]] = first[raw1]
    return keys.reshape(-1), vb, voff, seg_off


def test_config3_100k_storage_tries(khst, oracle):
    import torch
    from khipu_amd.device import Ctx
    rng = np.random.default_rng(3)
    ntries = 100_000
    keys, vb, voff, seg_off = storage_tries(rng, ntries)
    n = int(seg_off[-1])
    seg = np.repeat(np.arange(ntries, dtype=np.uint32), np.diff(seg_off).astype(np.int64))
    ctx = Ctx(0)
    dk, dv, do, ds = (torch.from_numpy(x).to("cuda:0") for x in (keys, vb, voff.astype(np.int64), seg))
    hh, ll, ii, st = ctx.build(dk, 32, dv, do, n, seg=ds, nseg=ntries, hash_keys=True)
    gpu = [hh[s].tobytes() if ll[s] else khst.EMPTY_TRIE_HASH for s in range(ntries)]
    cpu, cst = oracle.batch_roots(keys, (vb, voff), klen=32, seg_off=seg_off, hash_keys=True)
    assert gpu == cpu
    assert st.n_leaves == cst["distinct"] and st.n_node_hashes == cst["node_hashes"]
    # 17-bit segment prefix in the sort key; sampled tries against the sequential oracle
    for s in rng.choice(ntries, 12, replace=False):
        a, b = int(seg_off[s]), int(seg_off[s + 1])
        ks = [oracle.kec256(keys[32 * i:32 * i + 32].tobytes()) for i in range(a, b)]
        vs = [vb[int(voff[i]):int(voff[i + 1])].tobytes() for i in range(a, b)]
        assert gpu[s] == oracle.seq_root(ks, vs), s


@pytest.mark.parametrize("n", [1_000_000, 50_000_000], ids=["1m", "50m"])
def test_config2_block_commits(khst, oracle, n):
    """configs[2] (tests/blocks.py) at 1M and at its configured 50M resident accounts: 3 blocks of 20k dirty
    accounts (90% updates, 5% inserts, 5% deletes) and 2,000 resident 1k-slot storage tries
    with 10 dirty slots each (10% deletes), storage roots injected into the account bodies,
    one kh_block_commit per block.  Checks: every storage root against a from-scratch
    segmented GPU build and the CPU batch builder; sampled storage tries against the
    sequential oracle; the final state root against the CPU batch builder over the whole
    final state and a from-scratch GPU build."""
    import torch
    from khipu_amd.device import Ctx
    from tests.blocks import BlockWorkload
    ctx = Ctx(0)
    nb = 3
    w = BlockWorkload(ctx, n, nb)
    for b in range(nb):
        root = w.block(b)
    # storage tries
    K, V, O, T, N = w.final_storage()
    hh, ll, _, _ = ctx.build(K, 32, V, O, N, seg=T, nseg=w.nc, hash_keys=True)
    so = O.cpu().numpy().astype(np.uint64)
    tid = T.cpu().numpy()
    seg_off = np.searchsorted(tid, np.arange(w.nc + 1)).astype(np.uint64)
    kb = K.cpu().numpy()
    vb = V[:int(so[-1])].cpu().numpy()
    cpu, _ = oracle.batch_roots(kb, (vb, so), klen=32, seg_off=seg_off, hash_keys=True)
    for c in range(w.nc):
        assert w.roots[c] == hh[c].tobytes() == cpu[c], c
    for c in (0, 777, w.nc - 1):
        a, e = int(seg_off[c]), int(seg_off[c + 1])
        t = oracle.Trie()
        for i in range(a, e):
            t.put(oracle.kec256(kb[32 * i:32 * i + 32].tobytes()), vb[int(so[i]):int(so[i + 1])].tobytes())
        assert t.root_hash() == w.roots[c], c
    # storage-root injection (Account.withStateRoot, BlockWorldState.scala:243-248): every
    # contract body of the last block carries its CPU-built storage root in bytes
    # [len-65, len-33), every other byte is what the caller handed in
    _, a_vals, a_voff, cnt = w.ups[-1]
    av = a_vals.cpu().numpy()
    pv = w.ups_pristine[-1].cpu().numpy()
    ao = a_voff.cpu().numpy().astype(np.int64)
    expect = pv.copy()
    for c in range(w.nc):  # a_tid[c] = c (tests/blocks.py)
        e = int(ao[c + 1])
        assert av[e - 65:e - 33].tobytes() == cpu[c], c
        assert pv[e - 66] == 0xa0 and av[e - 66] == 0xa0
        expect[e - 65:e - 33] = np.frombuffer(cpu[c], np.uint8)
    assert (av[:int(ao[cnt])] == expect[:int(ao[cnt])]).all()
    # state trie: the committed state against a CPU batch build of the expected final state
    # (the bodies as handed in, contracts patched with the CPU storage roots)
    bodies = [torch.from_numpy(x.cpu().numpy()).to(x.device) for x in w.ups_pristine]
    bodies[-1] = torch.from_numpy(expect).to(bodies[-1].device)
    K, V, O, N = w.final_accounts(bodies=bodies)
    vo = O.cpu().numpy().astype(np.uint64)
    cpu, cst = oracle.batch_roots(K.cpu().numpy(), (V[:int(vo[-1])].cpu().numpy(), vo), klen=32, nthreads=16)
    assert cpu[0] == root
    assert len(w.state) == cst["distinct"]
    K, V, O, N = w.final_accounts()
    hf, _, _, _ = ctx.build(K, 32, V, O, N)
    assert hf[0].tobytes() == root
    # O(dirty) work: a block re-hashes a small fraction of the 1.36M nodes of a full build
    assert max(x[1] for x in w.t_commit) < 400_000, w.t_commit
