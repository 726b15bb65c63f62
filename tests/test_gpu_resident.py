"""GPU parity of the resident trie's incremental commit (kh_trie_open / kh_trie_apply,
SURVEY §8 f1) against the oracle trie folded put-by-put / remove-by-remove, and at
1M accounts against a from-scratch device build of the same final set."""
import random

import numpy as np
import pytest

from tests import cases as C
from tests.writeback import check_delta

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("sc", C.commit_scenarios(), ids=lambda s: s[0])
def test_commits_vs_oracle(khst, oracle, sc):
    from khipu_amd.device import Ctx, ResidentTrie
    name, ks, vs, batches = sc
    want = C.oracle_commits(oracle, ks, vs, batches)
    t = ResidentTrie(Ctx(0), ks, vs)
    assert t.root == want[0], name
    for i, (ups, dels) in enumerate(batches):
        assert t.commit(ups, dels) == want[i + 1], (name, i)
    t.close()


def test_commit_hash_keys(khst, oracle):
    """Addresses hashed on the device (KH_HASH_KEYS), as TrieAccounts keys them."""
    from khipu_amd.device import Ctx, ResidentTrie
    r = random.Random(8)
    addrs = [bytes(r.getrandbits(8) for _ in range(20)) for _ in range(500)]
    vals = [C.account_value(r) for _ in addrs]
    t = ResidentTrie(Ctx(0), addrs, vals, hash_keys=True)
    ups = [(a, C.account_value(r)) for a in r.sample(addrs, 40)] + [
        (bytes(r.getrandbits(8) for _ in range(20)), C.account_value(r)) for _ in range(10)]
    dels = r.sample(addrs, 15)
    got = t.commit(ups, dels, hash_keys=True)
    hk = [oracle.kec256(a) for a in addrs]
    want = C.oracle_commits(oracle, hk, vals, [([(oracle.kec256(a), v) for a, v in ups],
                                                [oracle.kec256(a) for a in dels])])
    assert t.root_hash == got
    assert got == want[1]


@pytest.mark.parametrize("klen", [135, 136, 300])
def test_commit_long_hashed_keys(khst, oracle, klen):
    """Keys hashed by the commit's key pass (k_f_keys_ck) at the one-block limit (135 bytes) and
    past it (the multi-block sponge): upserts and deletes hashed in the same launch, a delete of a
    key the same batch upserts (deletes apply after upserts), new keys and absent deletes."""
    from khipu_amd.device import Ctx, ResidentTrie
    r = random.Random(klen)
    keys = [bytes(r.getrandbits(8) for _ in range(klen)) for _ in range(400)]
    vals = [C.storage_value(r) for _ in keys]
    t = ResidentTrie(Ctx(0), keys, vals, hash_keys=True)
    ups = [(k, C.storage_value(r)) for k in r.sample(keys, 40)] + [
        (bytes(r.getrandbits(8) for _ in range(klen)), b"\x09") for _ in range(10)]
    dels = r.sample(keys, 25) + [ups[0][0], bytes(r.getrandbits(8) for _ in range(klen))]
    got = t.commit(ups, dels, hash_keys=True)
    want = C.oracle_commits(oracle, [oracle.kec256(k) for k in keys], vals,
                            [([(oracle.kec256(k), v) for k, v in ups], [oracle.kec256(k) for k in dels])])
    assert got == want[1]
    t.close()


def test_commit_uses_open_hash_keys(khst, oracle):
    """A storage trie opened with hash_keys=True hashes 32-byte slot keys on every commit
    without repeating the flag (the flag used to default to False); asking for
    the other encoder raises."""
    from khipu_amd.device import Ctx, ResidentTrie
    from khipu_amd._lib import MPTException
    r = random.Random(12)
    slots = [bytes(r.getrandbits(8) for _ in range(32)) for _ in range(300)]
    vals = [C.storage_value(r) for _ in slots]
    t = ResidentTrie(Ctx(0), slots, vals, hash_keys=True)
    ups = [(s, C.storage_value(r)) for s in r.sample(slots, 30)] + [
        (bytes(r.getrandbits(8) for _ in range(32)), b"\x07") for _ in range(5)]
    dels = r.sample(slots, 10)
    got = t.commit(ups, dels)
    want = C.oracle_commits(oracle, [oracle.kec256(s) for s in slots], vals,
                            [([(oracle.kec256(s), v) for s, v in ups], [oracle.kec256(s) for s in dels])])
    assert got == want[1]
    with pytest.raises(MPTException):
        t.commit(ups[:1], [], hash_keys=False)


def test_commit_1m_vs_full_build(khst):
    """configs[2]-style commit at 1M accounts: 20k dirty (90% updates, 5% inserts, 5%
    deletes) -> the root of a from-scratch build of the final set; only the changed
    paths are re-hashed."""
    import torch
    from khipu_amd.device import Ctx, ResidentTrie, _pack_dev
    ctx = Ctx(0)
    n = 1_000_000
    addr, vals, voff = ctx.synth_accounts(3, 0, n)
    keys = torch.empty(n * 32 + 64, dtype=torch.uint8, device="cuda:0")
    from khipu_amd._lib import check, lib
    from khipu_amd.device import _ptr
    torch.cuda.synchronize()
    check(lib().kh_dev_hash_keys(ctx.h, _ptr(addr), 20, n, _ptr(keys)))
    torch.cuda.synchronize()
    t = ResidentTrie.__new__(ResidentTrie)
    t.ctx, t.dev, t.h = ctx, "cuda:0", None
    t._open(keys, 32, vals, voff, n, False)
    r = random.Random(3)
    kh = keys[:32 * n].cpu().numpy().reshape(n, 32)
    vo = voff.cpu().numpy()
    vb = vals.cpu().numpy()
    state = {kh[i].tobytes(): vb[vo[i]:vo[i + 1]].tobytes() for i in range(n)}
    idx = r.sample(range(n), 19_000)
    ups = [(kh[i].tobytes(), C.account_value(r)) for i in idx[:18_000]]
    ups += [(bytes(r.getrandbits(8) for _ in range(32)), C.account_value(r)) for _ in range(1_000)]
    dels = [kh[i].tobytes() for i in idx[18_000:]]
    st = khst.KhStats()
    got = t.commit(ups, dels, stats=st)
    for k, v in ups:
        state[k] = v
    for k in dels:
        state.pop(k, None)
    fk = list(state.keys())
    kd, _ = _pack_dev(fk, "cuda:0")
    vd, od = _pack_dev([state[k] for k in fk], "cuda:0")
    hh, _, _, full = ctx.build(kd, 32, vd, od, len(fk))
    assert got == hh[0].tobytes()
    # ~19k changed leaves + the ~23k branches on their paths, not the 1.36M of a full build
    assert st.n_node_hashes < full.n_node_hashes // 20, (st.n_node_hashes, full.n_node_hashes)
    t.close()


@pytest.mark.parametrize("sc", C.commit_scenarios(), ids=lambda s: s[0])
def test_emit_nodes_after_commits(khst, oracle, sc):
    """kh_trie_emit_nodes is each commit's write-back DELTA: after open it is
    the oracle's reachable node set; after a block, (1) every emitted pair is an Updated entry
    of the faithful log of that block's puts/removes (MerklePatriciaTrie.scala:491-516), (2)
    every emitted node is reachable from the new root, and (3) every reachable node the store
    did not hold is emitted -- so the store after the hand-off holds the whole new trie."""
    from khipu_amd.device import Ctx, ResidentTrie
    name, ks, vs, batches = sc
    o = oracle.Trie()
    for k, v in zip(ks, vs):
        o.put(k, v)
    t = ResidentTrie(Ctx(0), ks, vs)
    store = dict(t.nodes())
    assert store == (o.reachable() if ks else {}), name
    o.persist().reopen()
    for i, (ups, dels) in enumerate(batches):
        for k, v in ups:
            o.put(k, v)
        for k in dels:
            o.remove(k)
        t.commit(ups, dels)
        delta = t.nodes()
        assert t.root == o.root_hash(), (name, i)
        want = o.reachable() if len(t) else {}
        upd = o.updated()
        assert all(h in upd and upd[h] == e for h, e in delta.items()), (name, i)
        assert all(h in want and want[h] == e for h, e in delta.items()), (name, i)
        missing = {h for h in want if h not in store and h not in delta}
        assert not missing, (name, i, len(missing))
        store.update(delta)
        o.persist().reopen()
    t.close()


def test_forest_vs_oracle(khst, oracle):
    """A forest (kh_forest_apply): storage tries of many contracts in one
    handle, blocks touching some of them; every touched trie's root equals the oracle's
    trie of that contract folded put-by-put / remove-by-remove; a trie deleted to empty has
    EMPTY_TRIE_HASH; identical keys in different tries stay apart.  The block's write-back
    delta (the storageNodeStorage.update half of BlockWorldState.scala:320-324) is held to
    the strict f2 contract (tests/writeback.py): every emitted pair an Updated entry of a
    touched trie's log, reachable from its new root, and no new reachable node missing."""
    from khipu_amd.device import Ctx, ResidentForest
    from tests.writeback import check_delta, settle
    r = random.Random(77)
    f = ResidentForest(Ctx(0), hash_keys=True, emit=True)
    tries = {}
    store = {}
    ids = [r.randrange(1 << 32) for _ in range(60)]
    for blk in range(8):
        ups, dels = [], []
        for t in r.sample(ids, 25):
            o = tries.setdefault(t, oracle.Trie())
            live = getattr(o, "_live", [])
            for _ in range(r.choice([1, 3, 10, 40])):
                slot = bytes(r.getrandbits(8) for _ in range(32)) if not live or r.random() < 0.6 else r.choice(live)
                ups.append((t, slot, C.storage_value(r)))
            if live and r.random() < 0.5:
                for slot in r.sample(live, min(len(live), r.choice([1, 5, len(live)]))):
                    dels.append((t, slot))
        if blk == 2:  # the same slot in two tries
            ups.append((ids[0], b"\x11" * 32, b"\x01"))
            ups.append((ids[1], b"\x11" * 32, b"\x02"))
        got = f.commit(ups, dels)
        for t, slot, v in ups:
            o = tries.setdefault(t, oracle.Trie())
            o.put(oracle.kec256(slot), v)
            o._live = list(dict.fromkeys(getattr(o, "_live", []) + [slot]))
        for t, slot in dels:
            tries[t].remove(oracle.kec256(slot))
            tries[t]._live = [s for s in tries[t]._live if s != slot]
        touched = {t for t, _, _ in ups} | {t for t, _ in dels}
        assert set(got) == touched, blk
        for t in touched:
            assert got[t] == tries[t].root_hash(), (blk, t)
        delta = f.nodes()
        check_delta(delta, [tries[t] for t in touched], store, ("forest block", blk))
        store.update(delta)
        settle(tries.values())
    f.close()


def test_forest_trie_id_bits(khst, oracle):
    """The forest's op sort takes the trie ids' bits from the ids committed before (so its
    32-bit prefix holds key bits too): small ids, then an id past the hint (the sort is redone
    with 32 bits), ids back inside it, many ops per trie (past the tie kernel's run limit when
    every op of a trie shared its prefix) and one slot in several tries; every root against
    the oracle's tries folded put by put."""
    from khipu_amd.device import Ctx, ResidentForest
    r = random.Random(5)
    f = ResidentForest(Ctx(0), hash_keys=True)
    tries = {}
    plan = [[0, 1, 2, 3], [1, 5, 7], [6, 5000, 3], [2, 4999, 5000, 70000], [0, 1, 65535, 7]]
    for blk, ids in enumerate(plan):
        ups = []
        for t in ids:
            for _ in range(r.choice([3, 90, 200])):
                ups.append((t, bytes(r.getrandbits(8) for _ in range(32)), C.storage_value(r)))
            ups.append((t, b"\x22" * 32, bytes([blk + 1])))
        dup = bytes(r.getrandbits(8) for _ in range(32))  # one key put twice: the later put wins
        ups += [(ids[0], dup, b"\x01"), (ids[0], dup, bytes([0x40 + blk]))]
        got = f.commit(ups, [])
        for t, slot, v in ups:
            tries.setdefault(t, oracle.Trie()).put(oracle.kec256(slot), v)
        assert set(got) == set(ids), blk
        for t in ids:
            assert got[t] == tries[t].root_hash(), (blk, t)
    f.close()


@pytest.mark.parametrize("hashed", [True, False], ids=["hashed", "raw"])
def test_forest_hot_trie(khst, oracle, hashed):
    """A forest whose ids span 2^16 (the op sort's short 24-bit composite form is in reach) with
    one hot contract taking ~4k slot writes per block beside ~1,500 one-op tries: the hot trie's
    run of equal sort prefixes is past the tie kernel's limit, so the sort widens (hashed keys)
    or never takes the short form (raw keys, whose structured leading bytes repeat); every root
    against the oracle's tries folded put by put."""
    from khipu_amd.device import Ctx, ResidentForest
    r = random.Random(11)
    f = ResidentForest(Ctx(0), hash_keys=hashed)
    tries = {}
    hot = 40000
    for blk in range(3):
        ups = []
        for t in r.sample(range(1 << 16), 1500):
            ups.append((t, bytes(r.getrandbits(8) for _ in range(32)), C.storage_value(r)))
        for i in range(4000):  # raw keys of the hot trie share their first 28 bytes
            slot = (bytes(28) + (blk * 4000 + i).to_bytes(4, "big")) if not hashed else bytes(r.getrandbits(8) for _ in range(32))
            ups.append((hot, slot, C.storage_value(r)))
        got = f.commit(ups, [])
        touched = set()
        for t, slot, v in ups:
            tries.setdefault(t, oracle.Trie()).put(oracle.kec256(slot) if hashed else slot, v)
            touched.add(t)
        assert set(got) == touched, blk
        for t in touched:
            assert got[t] == tries[t].root_hash(), (blk, t)
    f.close()


@pytest.mark.parametrize("case", ["repeat", "id_past_hint", "long_run"])
def test_forest_op_sort_edges_between_clean_blocks(khst, oracle, case):
    """The op sort's rare paths between ordinary blocks: a clean warm block, then a block with
    a key put twice (the later put wins), a trie id past the hinted bits (the sort redone with
    32), or a run of equal 24-bit sort prefixes past the tie kernel (the full sort, then the
    24-bit form off for 16 commits), then 18 clean blocks; every root against the oracle's
    tries folded put by put."""
    from khipu_amd.device import Ctx, ResidentForest
    r = random.Random(31 + ["repeat", "id_past_hint", "long_run"].index(case))
    f = ResidentForest(Ctx(0), hash_keys=True)
    tries = {}
    for blk in range(20):
        ids = r.sample(range(1, 1 << 15), 30)  # (ids of 17 hinted bits: the 24-bit sort form)
        ups = [(t, bytes(r.getrandbits(8) for _ in range(32)), C.storage_value(r)) for t in ids for _ in range(3)]
        if blk == 1 and case == "repeat":
            k = ups[5][1]
            ups.append((ups[5][0], k, b"\x7f"))
        if blk == 1 and case == "id_past_hint":
            ups.append((1 << 30, b"\x33" * 32, b"\x05"))
        if blk == 1 and case == "long_run":  # 12k ops in one trie: ~94 a run of the 24-bit prefix
            ups += [(7, bytes(r.getrandbits(8) for _ in range(32)), C.storage_value(r)) for _ in range(12000)]
        got = f.commit(ups, [])
        touched = set()
        for t, slot, v in ups:
            tries.setdefault(t, oracle.Trie()).put(oracle.kec256(slot), v)
            touched.add(t)
        assert set(got) == touched, blk
        for t in touched:
            assert got[t] == tries[t].root_hash(), (case, blk, t)
    f.close()


@pytest.mark.parametrize("sc", C.commit_scenarios()[:4], ids=lambda s: s[0])
def test_open_from_node_store(khst, oracle, sc):
    """kh_trie_open_nodes: a trie opened from its root hash and the
    oracle's persisted node store (MerklePatriciaTrie.apply(rootHash, source),
    MerklePatriciaTrie.scala:60-66,520-542) commits exactly like the oracle; a store
    missing a reachable node raises MPTNodeMissingException with that node's hash."""
    from khipu_amd.device import Ctx, ResidentTrie
    from khipu_amd._lib import MPTNodeMissingException
    name, ks, vs, batches = sc
    o = oracle.Trie()
    for k, v in zip(ks, vs):
        o.put(k, v)
    store = o.reachable() if ks else {}
    root = o.root_hash()
    t = ResidentTrie.from_nodes(Ctx(0), root, store)
    assert t.root == root and len(t) == len(set(ks)), name
    for i, (ups, dels) in enumerate(batches):
        for k, v in ups:
            o.put(k, v)
        for k in dels:
            o.remove(k)
        assert t.commit(ups, dels) == o.root_hash(), (name, i)
    t.close()
    if len(store) > 2:
        victim = sorted(store)[len(store) // 2]
        partial = {h: e for h, e in store.items() if h != victim}
        with pytest.raises(MPTNodeMissingException) as ei:
            ResidentTrie.from_nodes(Ctx(0), root, partial)
        assert ei.value.missing == victim


def test_open_from_node_store_1m(khst, oracle):
    """At 1M accounts: the node set a resident trie writes back at open, opened again from
    the root alone, gives the same roots through the same commits."""
    import torch
    from khipu_amd.device import Ctx, ResidentTrie
    ctx = Ctx(0)
    n = 1_000_000
    addr, vals, voff = ctx.synth_accounts(9, 0, n)
    a = ResidentTrie.__new__(ResidentTrie)
    a.ctx, a.dev, a.h = ctx, "cuda:0", None
    a._open(addr, 20, vals, voff, n, True)
    store = a.nodes()
    b = ResidentTrie.from_nodes(ctx, a.root, store, hash_keys=True)
    assert b.root == a.root and len(b) == n
    r = random.Random(5)
    ah = addr[:20 * n].view(n, 20).cpu().numpy()
    vo = voff.cpu().numpy()
    vb = vals.cpu().numpy()
    state = {ah[i].tobytes(): vb[vo[i]:vo[i + 1]].tobytes() for i in range(n)}
    for blk in range(3):
        ups = [(bytes(r.getrandbits(8) for _ in range(20)), C.account_value(r)) for _ in range(2000)]
        idx = r.sample(range(n), 500)
        ups += [(ah[i].tobytes(), C.account_value(r)) for i in idx[:400]]
        dels = [ah[i].tobytes() for i in idx[400:]]
        for k, v in ups:
            state[k] = v
        for k in dels:
            state.pop(k, None)
        want = oracle.batch_root(list(state.keys()), list(state.values()), klen=20, hash_keys=True)
        ra, rb = a.commit(ups, dels), b.commit(ups, dels)
        assert (ra == want, rb == want) == (True, True), blk
    a.close()
    b.close()


def test_block_commit_host_matches_device(khst):
    """kh_block_commit_host (host arrays, the JVM entry) against kh_block_commit (device
    tensors): a twin state trie + storage forest fed the same blocks gives the same state
    roots and the same storage roots."""
    import numpy as np
    from khipu_amd.device import Ctx, ResidentForest, ResidentTrie, block_commit_host
    from tests.blocks import BlockWorkload

    class Twin(BlockWorkload):
        def _commit(self, s_tid, s_keys, s_vals, s_voff, d_tid, d_keys, a_keys, a_vals, a_voff, a_tid, a_del,
                    timed=True):
            if not hasattr(self, "twin"):
                st = ResidentTrie.__new__(ResidentTrie)
                st.ctx, st.dev, st.h = self.ctx, self.dev, None
                st._open(self.keys, 32, self.vals, self.voff, self.n, False, emit=False)
                self.twin = (st, ResidentForest(self.ctx, hash_keys=True))
                self.twin_roots = []
            h = lambda t: None if t is None else t.cpu().numpy()  # noqa: E731
            args = [h(t) for t in (s_tid, s_keys, s_vals, s_voff, d_tid, d_keys, a_keys, a_vals, a_voff, a_tid,
                                   a_del)]
            root = super()._commit(s_tid, s_keys, s_vals, s_voff, d_tid, d_keys, a_keys, a_vals, a_voff, a_tid, a_del,
                                   timed)
            s_tid_h, s_keys_h, s_vals_h, s_voff_h, d_tid_h, d_keys_h, a_keys_h, a_vals_h, a_voff_h, a_tid_h, a_del_h = args
            n_s = len(s_tid_h)
            r2 = block_commit_host(self.twin[0], self.twin[1], s_tid_h.astype(np.uint32), s_keys_h, s_vals_h,
                                   s_voff_h[:n_s + 1].astype(np.uint64), None if d_tid_h is None else
                                   d_tid_h.astype(np.uint32), d_keys_h, a_keys_h, a_vals_h,
                                   a_voff_h[:len(a_tid_h) + 1].astype(np.uint64), a_tid_h.astype(np.uint32), a_del_h)
            assert r2 == root
            assert self.twin[1].last_roots() == self.forest.last_roots()
            return root

    ctx = Ctx(0)
    w = Twin(ctx, 30_000, 2, nc=40, ns=100, dirty=2_000)
    for b in range(2):
        w.block(b)


def test_host_handles_pair_on_the_shared_context(khst, oracle):
    """The JVM sequence of INTEGRATION.md: kh_trie_open_host + kh_forest_open(NULL) share
    the host entry points' context, so kh_block_commit_host accepts the pair."""
    import ctypes
    import random
    import numpy as np
    from khipu_amd import _lib
    from khipu_amd._lib import check, lib
    from khipu_amd.device import block_commit_host
    from khipu_amd import codec
    r = random.Random(21)
    keys = [bytes(r.getrandbits(8) for _ in range(32)) for _ in range(300)]
    vals = [codec.account_rlp(i, 10 ** 18 + i) for i in range(300)]
    kb = np.frombuffer(b"".join(keys), np.uint8)
    vb = np.frombuffer(b"".join(vals) + bytes(8), np.uint8)
    vo = np.concatenate([[0], np.cumsum([len(v) for v in vals])]).astype(np.uint64)
    root = np.zeros(32, np.uint8)
    st_h, fo_h = ctypes.c_void_p(), ctypes.c_void_p()
    check(lib().kh_trie_open_host(kb.ctypes.data, 32, vb.ctypes.data, vo.ctypes.data, 300, 0, root.ctypes.data,
                                  ctypes.byref(st_h)))
    check(lib().kh_forest_open(None, _lib.KH_HASH_KEYS, ctypes.byref(fo_h)))

    class H:  # the minimal handle shape block_commit_host needs
        def __init__(self, h):
            self.h = h
            self.ctx = type("C", (), {"_sync": staticmethod(lambda: None)})()
    state, forest = H(st_h), H(fo_h)
    # one slot in trie 0 for account 0 (its body gets the storage root), one plain update
    sk = np.frombuffer(bytes(31) + b"\x01", np.uint8)
    sv = np.frombuffer(b"\x05" + bytes(8), np.uint8)
    so = np.array([0, 1], np.uint64)
    ak = np.frombuffer(keys[0] + keys[1], np.uint8)
    bodies = [codec.account_rlp(1, 5), codec.account_rlp(2, 6)]
    av = np.frombuffer(b"".join(bodies) + bytes(8), np.uint8).copy()
    ao = np.array([0, len(bodies[0]), len(bodies[0]) + len(bodies[1])], np.uint64)
    at = np.array([0, _lib.KH_NO_TRIE], np.uint32)
    got = block_commit_host(state, forest, np.array([0], np.uint32), sk, sv, so, None, None, ak, av, ao, at, None)
    # expected: the oracle fold with the storage root written into account 0's body
    t = oracle.Trie()
    t.put(oracle.kec256(bytes(31) + b"\x01"), b"\x05")
    sroot = t.root_hash()
    b0 = bytearray(bodies[0])
    b0[len(b0) - 65:len(b0) - 33] = sroot
    exp_vals = [bytes(b0), bodies[1]] + vals[2:]
    assert got == oracle.seq_root(keys, exp_vals)
    lib().kh_trie_free(st_h)
    lib().kh_trie_free(fo_h)


def test_block_commit_refuses_non_account_body(khst, oracle):
    """An account upsert naming a storage trie whose body is not an account (no stateRoot
    field to write, Account.withStateRoot): kh_block_commit refuses the block with KH_EINVAL
    (the injection's error word is read with the account commit's first sync), the state
    trie unchanged -- the next block commits onto the old state as the oracle fold says."""
    import ctypes
    import random
    import numpy as np
    from khipu_amd import _lib
    from khipu_amd._lib import check, lib
    from khipu_amd.device import block_commit_host
    from khipu_amd import codec
    r = random.Random(22)
    keys = [bytes(r.getrandbits(8) for _ in range(32)) for _ in range(200)]
    vals = [codec.account_rlp(i, 10 ** 18 + i) for i in range(200)]
    kb = np.frombuffer(b"".join(keys), np.uint8)
    vb = np.frombuffer(b"".join(vals) + bytes(8), np.uint8)
    vo = np.concatenate([[0], np.cumsum([len(v) for v in vals])]).astype(np.uint64)
    root = np.zeros(32, np.uint8)
    st_h, fo_h = ctypes.c_void_p(), ctypes.c_void_p()
    check(lib().kh_trie_open_host(kb.ctypes.data, 32, vb.ctypes.data, vo.ctypes.data, 200, 0, root.ctypes.data,
                                  ctypes.byref(st_h)))
    check(lib().kh_forest_open(None, _lib.KH_HASH_KEYS, ctypes.byref(fo_h)))

    class H:
        def __init__(self, h):
            self.h = h
            self.ctx = type("C", (), {"_sync": staticmethod(lambda: None)})()
    state, forest = H(st_h), H(fo_h)
    sk = np.frombuffer(bytes(31) + b"\x02", np.uint8)
    sv = np.frombuffer(b"\x07" + bytes(8), np.uint8)
    so = np.array([0, 1], np.uint64)
    ak = np.frombuffer(keys[0], np.uint8)
    av = np.frombuffer(b"\x82\x01\x02" + bytes(8), np.uint8).copy()  # an RLP string, not an account
    ao = np.array([0, 3], np.uint64)
    at = np.array([0], np.uint32)
    with pytest.raises(Exception, match="not an account body"):
        block_commit_host(state, forest, np.array([0], np.uint32), sk, sv, so, None, None, ak, av, ao, at, None)
    # the next block: a plain account update onto the unchanged state
    body = codec.account_rlp(9, 99)
    got = block_commit_host(state, forest, None, None, None, None, None, None, np.frombuffer(keys[1], np.uint8),
                            np.frombuffer(body + bytes(8), np.uint8).copy(), np.array([0, len(body)], np.uint64),
                            np.array([_lib.KH_NO_TRIE], np.uint32), None)
    assert got == oracle.seq_root(keys, [vals[0], body] + vals[2:])
    lib().kh_trie_free(st_h)
    lib().kh_trie_free(fo_h)


def _pair(r):
    """Two keys sharing 63 nibbles: they hang under a depth-63 branch, their leaves' paths empty."""
    k1 = bytearray(C._rk(r))
    k2 = bytearray(k1)
    k2[31] ^= 0x01
    return bytes(k1), bytes(k2)


@pytest.mark.parametrize("small", [False, True], ids=["hashed", "inline"])
def test_value_only_branch_vs_oracle(khst, oracle, small):
    """khipu's value-only branch (forest.h VB_DEPTH): a re-put of a key whose leaf hangs under
    a depth-63 branch goes through putInLeafNode with ml == 0 and an empty existing key and
    leaves a childless branch holding the new value (MerklePatriciaTrie.scala:187-199 ->
    putInBranchNode :258-262; tests/test_oracle.py pins the shape).  Every block equals the
    oracle's fold and its write-back delta the oracle's Updated log (tests/writeback.py):
    making it, updating it, its sibling removed (an extension above it, then merged with the
    one above that), a new branch above it, get() of its key; removing its key is refused like
    khipu's MPTException ("Branch with no subvalues") with the trie unchanged; a node store of
    every emitted node reopens it (kh_trie_open_nodes).  small: 1-byte values (the branch is
    embedded in its parent, < 32 B) instead of account bodies."""
    from khipu_amd.device import Ctx, ResidentTrie
    from khipu_amd._lib import MPTException
    r = random.Random(64 if small else 63)
    val = (lambda: bytes([r.randrange(1, 0x80)])) if small else (lambda: C.account_value(r))
    k1, k2 = _pair(r)
    k3 = bytearray(k1)
    k3[31] = (k3[31] & 0x0F) | (((k3[31] >> 4) ^ 0x3) << 4)  # 62 nibbles shared with k1 and k2
    k3 = bytes(k3)
    q1, q2 = _pair(r)  # a second pair whose value-only branch is made and kept
    others = [C._rk(r) for _ in range(300)]
    ks = others + [k1, k2, q1, q2]
    vs = [val() for _ in ks]
    o = oracle.Trie()
    for k, v in zip(ks, vs):
        o.put(k, v)
    ctx = Ctx(0)
    t = ResidentTrie(ctx, ks, vs)
    assert t.root == o.root_hash()
    store = dict(t.nodes())
    o.persist().reopen()
    live = dict(zip(ks, vs))

    def block(ups, dels, what):
        for k, v in ups:
            o.put(k, v)
            live[k] = v
        for k in dels:
            o.remove(k)
            live.pop(k, None)
        root = t.commit(ups, dels)
        assert root == o.root_hash(), what
        delta = t.nodes()
        check_delta(delta, [o], store, what)
        store.update(delta)
        o.persist().reopen()
        probe = [k1, k2, k3, q1, q2] + others[:20]
        assert t.get(probe) == [live.get(k) for k in probe], what

    block([(k1, val()), (others[0], val()), (q1, val())], [], "value-only branches made")
    block([(k1, val())], [others[1]], "value-only branch updated")
    size = len(t)
    with pytest.raises(MPTException, match="value-only branch"):
        t.commit([(others[2], val())], [k1])
    assert t.get_root() == o.root_hash() and len(t) == size
    block([(others[3], val())], [k2], "its sibling removed: an extension above it")
    block([(k3, val())], [], "a new branch above it")
    block([(k1, val()), (q1, val())], [others[4]], "updated under the new branch")
    block([], [k3], "the branch above it removed again")
    # reopen from the node store: the value-only branches decode into records
    t2 = ResidentTrie.from_nodes(ctx, t.root, store)
    assert t2.root == t.root and len(t2) == len(t)
    probe = [k1, q1, q2] + others[:10]
    assert t2.get(probe) == [live.get(k) for k in probe]
    v = val()
    o.put(q1, v)
    assert t2.commit([(q1, v)], []) == o.root_hash()
    t2.close()
    t.close()


def test_value_only_branch_in_block_commit(khst, oracle):
    """kh_block_commit with value-only branches made in both phases of one block: in a storage
    trie (raw slot keys) and in the state trie, whose account phase runs beside the storage
    phase and reads its values only after the storage roots are injected (the branch's
    encoding needs them).  Two blocks; the state root equals the oracle's fold with the
    injected storageRoot, the storage root the oracle's."""
    import ctypes
    from khipu_amd import _lib, codec
    from khipu_amd._lib import check, lib
    from khipu_amd.device import block_commit_host
    r = random.Random(66)
    a1, a2 = _pair(r)
    s1, s2 = _pair(r)
    akeys = [C._rk(r) for _ in range(300)] + [a1, a2]
    avals = [codec.account_rlp(i, 10 ** 18 + i) for i in range(len(akeys))]
    kb = np.frombuffer(b"".join(akeys), np.uint8)
    vb = np.frombuffer(b"".join(avals) + bytes(8), np.uint8)
    vo = np.concatenate([[0], np.cumsum([len(v) for v in avals])]).astype(np.uint64)
    root = np.zeros(32, np.uint8)
    st_h, fo_h = ctypes.c_void_p(), ctypes.c_void_p()
    check(lib().kh_trie_open_host(kb.ctypes.data, 32, vb.ctypes.data, vo.ctypes.data, len(akeys), 0,
                                  root.ctypes.data, ctypes.byref(st_h)))
    check(lib().kh_forest_open(None, 0, ctypes.byref(fo_h)))

    class H:
        def __init__(self, h):
            self.h = h
            self.ctx = type("C", (), {"_sync": staticmethod(lambda: None)})()
    state, forest = H(st_h), H(fo_h)
    so_t = oracle.Trie()  # storage trie 0
    st_t = oracle.Trie()  # the state trie
    for k, v in zip(akeys, avals):
        st_t.put(k, v)
    slots = [C._rk(r) for _ in range(40)] + [s1, s2]

    def block(sups, aups):
        for k, v in sups:
            so_t.put(k, v)
        sroot = so_t.root_hash()
        sk = np.frombuffer(b"".join(k for k, _ in sups), np.uint8)
        sv = np.frombuffer(b"".join(v for _, v in sups) + bytes(8), np.uint8)
        so = np.concatenate([[0], np.cumsum([len(v) for _, v in sups])]).astype(np.uint64)
        bodies = [codec.account_rlp(n, b) for _, (n, b) in aups]
        av = np.frombuffer(b"".join(bodies) + bytes(8), np.uint8).copy()
        ao = np.concatenate([[0], np.cumsum([len(b) for b in bodies])]).astype(np.uint64)
        at = np.array([0] + [_lib.KH_NO_TRIE] * (len(aups) - 1), np.uint32)  # the first names trie 0
        ak = np.frombuffer(b"".join(k for k, _ in aups), np.uint8)
        got = block_commit_host(state, forest, np.zeros(len(sups), np.uint32), sk, sv, so, None, None, ak, av, ao,
                                at, None)
        b0 = bytearray(bodies[0])
        b0[len(b0) - 65:len(b0) - 33] = sroot
        for (k, _), b in zip(aups, [bytes(b0)] + bodies[1:]):
            st_t.put(k, b)
        assert got == st_t.root_hash()

    block([(k, bytes([r.randrange(1, 256)]) * r.choice([1, 3, 33])) for k in slots],
          [(akeys[0], (1, 5)), (akeys[1], (2, 6))])
    # the second block re-puts s1 (a storage value-only branch) and a1 (a state one, naming trie 0)
    block([(s1, b"\x07" * 33), (slots[0], b"\x09")], [(a1, (3, 7)), (akeys[2], (4, 8))])
    block([(s1, b"\x08"), (slots[1], b"\x0a" * 5)], [(a1, (5, 9))])
    lib().kh_trie_free(st_h)
    lib().kh_trie_free(fo_h)


def test_value_only_branch_versions_and_compaction(khst, oracle):
    """A value-only branch through a savepoint (rolled back, then made again), a copy, and a
    compaction (its value moves to the dense heap): roots and get() stay the oracle's."""
    from khipu_amd.device import Ctx, ResidentTrie
    r = random.Random(65)
    k1, k2 = _pair(r)
    others = [C._rk(r) for _ in range(100)]
    ks = others + [k1, k2]
    vs = [C.account_value(r) for _ in ks]
    o = oracle.Trie()
    for k, v in zip(ks, vs):
        o.put(k, v)
    t = ResidentTrie(Ctx(0), ks, vs)
    parent = t.root
    t.savepoint()
    t.commit([(k1, C.account_value(r))], [])
    t.rollback()
    assert t.get_root() == parent == o.root_hash()
    v1 = C.account_value(r)
    o.put(k1, v1)
    assert t.commit([(k1, v1)], []) == o.root_hash()
    c = t.copy()
    t.compact()
    assert t.get_root() == o.root_hash() and t.get([k1, k2]) == [v1, vs[-1]]
    v2 = C.account_value(r)
    o.put(k1, v2)
    o.remove(others[0])
    assert t.commit([(k1, v2)], [others[0]]) == o.root_hash()
    assert c.get([k1]) == [v1]
    c.close()
    t.close()


@pytest.mark.parametrize("sc", C.commit_scenarios()[:4] + C.commit_scenarios()[5:6], ids=lambda s: s[0])
def test_batched_get_vs_oracle(khst, oracle, sc):
    """kh_trie_get (MerklePatriciaTrie.get, MerklePatriciaTrie.scala:90-147) after open and
    after every commit: every key ever put (present, updated, or removed by the last commit),
    absent keys sharing long prefixes with present ones (they end inside an extension or at
    an empty branch slot), and inline leaves of the storage / deep tries."""
    from khipu_amd.device import Ctx, ResidentTrie
    name, ks, vs, batches = sc
    r = random.Random(17)
    o = oracle.Trie()
    for k, v in zip(ks, vs):
        o.put(k, v)
    t = ResidentTrie(Ctx(0), ks, vs)
    seen = list(ks)

    def probes():
        near = []
        for k in r.sample(seen, min(20, len(seen))):
            b = bytearray(k)
            b[r.randrange(32)] ^= 1 << r.randrange(8)
            near.append(bytes(b))
            b = bytearray(k)
            b[31] ^= 0x01  # shares 63 nibbles
            near.append(bytes(b))
        return list(dict.fromkeys(seen + near + [C._rk(r) for _ in range(10)]))

    q = probes()
    assert t.get(q) == [o.get(k) for k in q], name
    for ups, dels in batches:
        for k, v in ups:
            o.put(k, v)
        for k in dels:
            o.remove(k)
        t.commit(ups, dels)
        seen += [k for k, _ in ups]
        q = probes()
        assert t.get(q) == [o.get(k) for k in q], name
    assert t.get([]) == []
    t.close()


def test_batched_get_hash_keys_and_forest(khst, oracle):
    """Raw keys on a KH_HASH_KEYS trie (hashed on the device, as its commits are), and a
    forest answering (trie id, key) queries, including ids of tries it does not hold."""
    from khipu_amd.device import Ctx, ResidentForest, ResidentTrie
    r = random.Random(23)
    ctx = Ctx(0)
    addrs = [bytes(r.getrandbits(8) for _ in range(20)) for _ in range(300)]
    vals = [C.account_value(r) for _ in addrs]
    t = ResidentTrie(ctx, addrs, vals, hash_keys=True)
    t.commit([(addrs[0], b"\x01" * 70)], addrs[1:3], hash_keys=True)
    want = [b"\x01" * 70, None, None] + vals[3:] + [None]
    assert t.get(addrs + [bytes(20)]) == want
    t.close()
    f = ResidentForest(ctx)
    tries = {tid: {C._rk(r): C.storage_value(r) for _ in range(r.randrange(1, 60))} for tid in (3, 7, 1000)}
    f.commit([(tid, k, v) for tid, kv in tries.items() for k, v in kv.items()])
    q = [(tid, k) for tid, kv in tries.items() for k in kv] + [(5, next(iter(tries[3])))] + [(7, C._rk(r))]
    assert f.get(q) == [tries.get(tid, {}).get(k) for tid, k in q]
    f.close()
