"""GPU parity of versioned resident commits and of kh_block_commit's
write-back deltas (f2), against the khipu-faithful oracle.

Reference behaviour mirrored:
- Ledger.executeBlock flushes the parallel attempt, and when its root does not validate it
  re-executes sequentially from the SAME parent state (khipu-eth/.../ledger/Ledger.scala:237-271);
  validateBlockAfterExecution rejects a block (:603-620) -> kh_trie_savepoint / kh_trie_rollback;
- TrieAccounts.rootHash flushes a COPY and leaves the trie untouched (TrieAccounts.scala:73-80,
  MerklePatriciaTrie.copy :556) -> kh_trie_root_of, kh_trie_copy;
- BlockWorldState.persist hands the storage tries' and the account trie's Updated nodes to
  their node storages (BlockWorldState.scala:312-330) -> kh_trie_emit_nodes on both handles
  of kh_block_commit, held to tests/writeback.py's strict contract.
"""
import random

import numpy as np
import pytest

from tests import cases as C
from tests.writeback import check_delta, reachable, settle

pytestmark = pytest.mark.gpu


def _oracle(oracle, ks, vs):
    o = oracle.Trie()
    for k, v in zip(ks, vs):
        o.put(k, v)
    return o


def _fold(o, ups, dels):
    for k, v in ups:
        o.put(k, v)
    for k in dels:
        o.remove(k)
    return o.root_hash()


@pytest.mark.parametrize("sc", C.commit_scenarios()[:4] + C.commit_scenarios()[6:], ids=lambda s: s[0])
def test_rollback_then_retry(khst, oracle, sc):
    """Ledger.scala:237-271: a block committed, rolled back, and a DIFFERENT block committed
    from the same parent equals the oracle fold from the parent; after the rollback the root,
    get() answers, size and write-back set are the parent's."""
    from khipu_amd.device import Ctx, ResidentTrie
    name, ks, vs, batches = sc
    r = random.Random(5)
    t = ResidentTrie(Ctx(0), ks, vs)
    parent_nodes = t.nodes()
    o = _oracle(oracle, ks, vs)
    parent = o.root_hash()
    assert t.root == parent
    probe = list(ks[:50]) + [k for b in batches for k, _ in b[0]][:50]
    parent_get = t.get(probe) if probe else []
    for i, (ups, dels) in enumerate(batches):
        assert t.savepoint() == 1
        attempt = [(k, C.account_value(r)) for k, _ in ups] + [(C._rk(r), C.account_value(r)) for _ in range(3)]
        t.commit(attempt, dels[::2])
        t.rollback()
        assert t.savepoint_depth() == 0
        assert t.root == parent and t.get_root() == parent, (name, i)
        if probe:
            assert t.get(probe) == parent_get, (name, i)
        if i == 0:
            assert len(t) == len(set(ks)), name
        assert t.nodes() == parent_nodes, (name, i)
        # the sequential retry: the real batch from the parent
        want = _fold(o, ups, dels)
        assert t.commit(ups, dels) == want, (name, i)
        parent = want
        parent_nodes = t.nodes()
        parent_get = t.get(probe) if probe else []
    t.close()


def test_nested_savepoints_and_multi_commit(khst, oracle):
    """Savepoints nest: commits under the inner one roll back to it, the outer one still
    returns to its own version; several commits under one savepoint undo together; release
    keeps the commits (and the outer savepoint can still undo them)."""
    from khipu_amd.device import Ctx, ResidentTrie
    r = random.Random(9)
    ks = [C._rk(r) for _ in range(3000)]
    vs = [C.account_value(r) for _ in ks]
    t = ResidentTrie(Ctx(0), ks, vs)
    o = _oracle(oracle, ks, vs)
    r0 = o.root_hash()

    def batch(n_up, n_new, n_del):
        ups = [(k, C.account_value(r)) for k in r.sample(ks, n_up)] + [(C._rk(r), C.account_value(r))
                                                                         for _ in range(n_new)]
        return ups, r.sample(ks, n_del)

    b1, b2, b3, b4 = batch(100, 20, 30), batch(50, 50, 10), batch(10, 500, 200), batch(70, 5, 5)
    assert t.savepoint() == 1
    t.commit(*b1)
    r1 = oracle.seq_root(*_kv_after(ks, vs, [b1]))
    assert t.root == r1
    assert t.savepoint() == 2
    t.commit(*b2)
    t.commit(*b3)
    t.rollback()                       # back to after b1
    assert t.root == r1 and t.get_root() == r1
    assert t.savepoint() == 2
    t.commit(*b4)
    t.release()                        # keep b4: depth 1
    r14 = oracle.seq_root(*_kv_after(ks, vs, [b1, b4]))
    assert t.root == r14 and t.savepoint_depth() == 1
    t.rollback()                       # the outer savepoint: before b1
    assert t.root == r0 and len(t) == len(ks)
    assert t.commit(*b3) == oracle.seq_root(*_kv_after(ks, vs, [b3]))
    t.close()


def _kv_after(ks, vs, batches):
    """(keys, vals) of the state after the batches (upserts then deletes each), in put order."""
    state = dict(zip(ks, vs))
    for ups, dels in batches:
        for k, v in ups:
            state[k] = v
        for k in dels:
            state.pop(k, None)
    return list(state.keys()), list(state.values())


def test_rollback_across_map_rebuild(khst, oracle):
    """A commit that outgrows the anchor map (a rebuild voids the slot log) still rolls back:
    the map is rebuilt from the restored records; later commits match the oracle."""
    from khipu_amd.device import Ctx, ResidentTrie
    r = random.Random(10)
    ks = [C._rk(r) for _ in range(200)]
    vs = [C.account_value(r) for _ in ks]
    t = ResidentTrie(Ctx(0), ks, vs)
    o = _oracle(oracle, ks, vs)
    parent = o.root_hash()
    t.savepoint()
    big = [(C._rk(r), C.account_value(r)) for _ in range(20_000)]  # 100x the trie: the map grows
    t.commit(big, ks[:50])
    t.rollback()
    assert t.root == parent and t.get(ks[:60]) == vs[:60]
    ups = [(k, C.account_value(r)) for k in ks[100:140]] + [(C._rk(r), C.account_value(r)) for _ in range(40)]
    assert t.commit(ups, ks[:10]) == _fold(o, ups, ks[:10])
    t.close()


@pytest.mark.parametrize("sc", C.commit_scenarios()[:3], ids=lambda s: s[0])
def test_root_of_leaves_trie_unchanged(khst, oracle, sc):
    """kh_trie_root_of = TrieAccounts.rootHash: the root of a copy flushed with the batch,
    the trie (root, get, write-back set) unchanged; the same batch committed gives that root."""
    from khipu_amd.device import Ctx, ResidentTrie
    name, ks, vs, batches = sc
    t = ResidentTrie(Ctx(0), ks, vs)
    o = _oracle(oracle, ks, vs)
    for i, (ups, dels) in enumerate(batches):
        before, nodes = t.root, t.nodes()
        spec = t.root_of(ups, dels)
        assert t.get_root() == before and t.nodes() == nodes and t.savepoint_depth() == 0, (name, i)
        want = _fold(o, ups, dels)
        assert spec == want, (name, i)
        assert t.commit(ups, dels) == want, (name, i)
    t.close()


def test_copy_is_independent(khst, oracle):
    """kh_trie_copy = MerklePatriciaTrie.copy: the copy and the original take different
    commits; each matches its own oracle fold."""
    from khipu_amd.device import Ctx, ResidentTrie
    r = random.Random(11)
    ks = [C._rk(r) for _ in range(1500)]
    vs = [C.account_value(r) for _ in ks]
    t = ResidentTrie(Ctx(0), ks, vs)
    u = t.copy()
    assert u.root == t.root and len(u) == len(t)
    oa, ob = _oracle(oracle, ks, vs), _oracle(oracle, ks, vs)
    for _ in range(3):
        ua = [(k, C.account_value(r)) for k in r.sample(ks, 40)] + [(C._rk(r), C.account_value(r)) for _ in range(9)]
        ub = [(k, C.account_value(r)) for k in r.sample(ks, 40)]
        da, db = r.sample(ks, 7), r.sample(ks, 11)
        assert t.commit(ua, da) == _fold(oa, ua, da)
        assert u.commit(ub, db) == _fold(ob, ub, db)
    assert t.get(ks[:200]) == [oa.get(k) for k in ks[:200]]
    assert u.get(ks[:200]) == [ob.get(k) for k in ks[:200]]
    t.close()
    u.close()


def test_forest_rollback(khst, oracle):
    """A forest (storage tries) rolls back too: the touched tries' roots, get() answers and
    kh_forest_last_roots are the parent's; the retry matches the oracle per trie."""
    from khipu_amd.device import Ctx, ResidentForest
    r = random.Random(12)
    f = ResidentForest(Ctx(0), hash_keys=True)
    tries = {t: {C._rk(r): C.storage_value(r) for _ in range(r.randrange(1, 80))} for t in range(30)}
    f.commit([(t, k, v) for t, kv in tries.items() for k, v in kv.items()])
    last = f.last_roots()
    q = [(t, k) for t, kv in tries.items() for k in list(kv)[:5]]
    before = f.get(q)
    f.savepoint()
    f.commit([(t, C._rk(r), b"\x09") for t in range(0, 30, 2)], [(t, next(iter(tries[t]))) for t in range(1, 30, 3)])
    f.rollback()
    assert f.last_roots() == last and f.get(q) == before
    ups = [(t, C._rk(r), C.storage_value(r)) for t in range(5, 25)]
    dels = [(t, k) for t in range(0, 10) for k in list(tries[t])[:2]]
    got = f.commit(ups, dels)
    for t, k, v in ups:
        tries[t][k] = v
    for t, k in dels:
        tries[t].pop(k, None)
    for t in got:
        o = oracle.Trie()
        for k, v in tries[t].items():
            o.put(oracle.kec256(k), v)
        assert got[t] == o.root_hash(), t
    f.close()


def _host_pair(khst, n, seed):
    """A state trie (kh_trie_open_host) and a forest on the shared context, as the JVM opens them."""
    import ctypes
    from khipu_amd import _lib, codec
    from khipu_amd._lib import check, lib
    r = random.Random(seed)
    keys = [bytes(r.getrandbits(8) for _ in range(32)) for _ in range(n)]
    vals = [codec.account_rlp(i, 10 ** 18 + i) for i in range(n)]
    kb = np.frombuffer(b"".join(keys), np.uint8)
    vb = np.frombuffer(b"".join(vals) + bytes(8), np.uint8)
    vo = np.concatenate([[0], np.cumsum([len(v) for v in vals])]).astype(np.uint64)
    root = np.zeros(32, np.uint8)
    st_h, fo_h = ctypes.c_void_p(), ctypes.c_void_p()
    check(lib().kh_trie_open_host(kb.ctypes.data, 32, vb.ctypes.data, vo.ctypes.data, n, _lib.KH_EMIT_NODES,
                                  root.ctypes.data, ctypes.byref(st_h)))
    check(lib().kh_forest_open(None, _lib.KH_HASH_KEYS | _lib.KH_EMIT_NODES, ctypes.byref(fo_h)))
    from khipu_amd.device import ResidentForest, ResidentTrie

    class Ctx0:
        device = 0

        @staticmethod
        def _sync():
            pass
    state = ResidentTrie.__new__(ResidentTrie)
    state.ctx, state.dev, state.h, state.hash_keys, state.root = Ctx0, "cuda:0", st_h, False, root.tobytes()
    forest = ResidentForest.__new__(ResidentForest)
    forest.ctx, forest.dev, forest.h, forest.hash_keys = Ctx0, "cuda:0", fo_h, True
    return keys, vals, state, forest


def test_refused_block_leaves_both_handles_at_parent(khst, oracle):
    """kh_block_commit is all or nothing: an account upsert naming a storage trie
    whose body is not an account is refused AFTER the storage phase ran; both handles are
    rolled back -- the forest's roots, slots, last roots and write-back set, and the state
    trie's root and write-back set are the parent's -- and the next block commits onto the
    parent as the oracle fold says."""
    from khipu_amd import _lib, codec
    from khipu_amd.device import block_commit_host
    keys, vals, state, forest = _host_pair(khst, 200, 22)
    # block 1 (accepted): slot 1 of trie 0, account 0 carries its storage root
    sk1 = np.frombuffer(bytes(31) + b"\x01", np.uint8)
    body0 = codec.account_rlp(1, 5)
    av = np.frombuffer(body0 + bytes(8), np.uint8).copy()
    block_commit_host(state, forest, np.array([0], np.uint32), sk1, np.frombuffer(b"\x05" + bytes(8), np.uint8),
                      np.array([0, 1], np.uint64), None, None, np.frombuffer(keys[0], np.uint8), av,
                      np.array([0, len(body0)], np.uint64), np.array([0], np.uint32), None)
    parent_state, parent_last = state.get_root(), forest.last_roots()
    parent_snodes, parent_fnodes = state.nodes(), forest.nodes()
    parent_get = forest.get([(0, bytes(31) + b"\x01"), (0, bytes(31) + b"\x02"), (7, bytes(31) + b"\x02")])
    # block 2 (refused in the account phase): slots into tries 0 and 7, a bad body for trie 7
    sk = np.frombuffer(bytes(31) + b"\x02" + bytes(31) + b"\x02", np.uint8)
    bad = np.frombuffer(b"\x82\x01\x02" + bytes(8), np.uint8).copy()
    with pytest.raises(Exception, match="not an account body"):
        block_commit_host(state, forest, np.array([0, 7], np.uint32), sk, np.frombuffer(b"\x07\x08" + bytes(8), np.uint8),
                          np.array([0, 1, 2], np.uint64), None, None, np.frombuffer(keys[1], np.uint8), bad,
                          np.array([0, 3], np.uint64), np.array([7], np.uint32), None)
    assert state.get_root() == parent_state
    assert forest.last_roots() == parent_last
    assert forest.get([(0, bytes(31) + b"\x01"), (0, bytes(31) + b"\x02"), (7, bytes(31) + b"\x02")]) == parent_get
    assert state.nodes() == parent_snodes and forest.nodes() == parent_fnodes
    assert state.savepoint_depth() == 0 and forest.savepoint_depth() == 0
    # block 3: a plain account update onto the parent
    body = codec.account_rlp(9, 99)
    got = block_commit_host(state, forest, None, None, None, None, None, None, np.frombuffer(keys[1], np.uint8),
                            np.frombuffer(body + bytes(8), np.uint8).copy(), np.array([0, len(body)], np.uint64),
                            np.array([_lib.KH_NO_TRIE], np.uint32), None)
    t = oracle.Trie()
    t.put(oracle.kec256(bytes(31) + b"\x01"), b"\x05")
    b0 = bytearray(body0)
    b0[len(b0) - 65:len(b0) - 33] = t.root_hash()
    assert got == oracle.seq_root(keys, [bytes(b0), body] + vals[2:])
    state.close()
    forest.close()


def test_refused_account_descent_rolls_back_storage(khst, oracle):
    """The account phase's own refusal (removing a key held by khipu's value-only branch: its
    fix throws MPTException("Branch with no subvalues"), MerklePatriciaTrie.scala:323-370,
    430-477) comes after the storage phase: the forest is rolled back with the state trie."""
    from khipu_amd import codec
    from khipu_amd.device import block_commit_host
    keys, vals, state, forest = _host_pair(khst, 150, 23)
    k1 = bytearray(keys[0])
    k1[31] ^= 0x01  # 63 nibbles shared with keys[0]
    body = codec.account_rlp(3, 3)
    nt = np.array([0xFFFFFFFF], np.uint32)
    # put k1 (a sibling of keys[0] under a depth-63 branch), then re-put keys[0]: its leaf
    # (remaining path empty) becomes a value-only branch
    for k in (bytes(k1), keys[0]):
        block_commit_host(state, forest, None, None, None, None, None, None, np.frombuffer(k, np.uint8),
                          np.frombuffer(body + bytes(8), np.uint8).copy(), np.array([0, len(body)], np.uint64),
                          nt, None)
    parent_state, parent_last = state.get_root(), forest.last_roots()
    sk = np.frombuffer(bytes(31) + b"\x03", np.uint8)
    with pytest.raises(Exception, match="value-only branch"):
        block_commit_host(state, forest, np.array([5], np.uint32), sk, np.frombuffer(b"\x11" + bytes(8), np.uint8),
                          np.array([0, 1], np.uint64), None, None, np.frombuffer(keys[1], np.uint8),
                          np.frombuffer(body + bytes(8), np.uint8).copy(), np.array([0, len(body)], np.uint64),
                          nt, np.frombuffer(keys[0], np.uint8))
    assert state.get_root() == parent_state and forest.last_roots() == parent_last
    assert forest.get([(5, bytes(31) + b"\x03")]) == [None]
    assert state.get([keys[0]]) == [body]
    state.close()
    forest.close()


def test_block_rollback_and_sequential_retry(khst, oracle):
    """Ledger.executeBlock's retry: savepoints on both handles, the parallel attempt's block
    committed and rolled back, the sequential block committed from the parent: its state root
    and storage roots equal a fresh build of the retried block's final state."""
    import torch
    from khipu_amd.device import Ctx
    from tests.blocks import BlockWorkload
    ctx = Ctx(0)
    w = BlockWorkload(ctx, 60_000, 2, nc=30, ns=200, dirty=3_000)
    w.block(0)
    parent_root, parent_last = w.state.get_root(), w.forest.last_roots()
    w.state.savepoint()
    w.forest.savepoint()
    ops = w.prepare(1)
    attempt = list(ops)
    attempt[7] = ops[7].clone()  # the attempt's account bodies (patched in place by the commit)
    attempt[2] = ops[2].clone()
    attempt[2][:ops[2].numel() - 64] ^= 0x5A  # a different storage outcome: other slot values
    from khipu_amd.device import block_commit
    from khipu_amd._lib import KhStats
    s_tid, s_keys, s_vals, s_voff, d_tid, d_keys, a_keys, a_vals, a_voff, a_tid, a_del = attempt
    block_commit(w.state, w.forest, s_tid, s_keys, s_vals, s_voff, s_tid.numel(), d_tid, d_keys, d_tid.numel(),
                 a_keys, a_vals, a_voff, a_tid, a_tid.numel(), a_del, a_del.numel() // 32, stats=KhStats())
    w.state.rollback()
    w.forest.rollback()
    assert w.state.get_root() == parent_root and w.forest.last_roots() == parent_last
    root = w.commit_prepared(ops)
    K, V, O, N = w.final_accounts()
    hf, _, _, _ = ctx.build(K, 32, V, O, N)
    assert hf[0].tobytes() == root
    K, V, O, T, N = w.final_storage()
    hh, ll, _, _ = ctx.build(K, 32, V, O, N, seg=T, nseg=w.nc, hash_keys=True)
    for c in range(w.nc):
        assert w.roots[c] == hh[c].tobytes(), c
    torch.cuda.synchronize()


def test_block_commit_write_back_deltas(khst, oracle):
    """kh_block_commit's two write-back deltas (BlockWorldState.scala:312-330: the storage tries
    to storageNodeStorage, the account trie to accountNodeStorage), block by block, against the
    oracle's Updated logs and reachable sets (tests/writeback.py): the storage forest's delta
    over the touched contracts' tries, the state trie's over the account trie with the injected
    storage roots in the contract bodies."""
    import torch
    from khipu_amd.device import Ctx
    from tests.blocks import BlockWorkload
    ctx = Ctx(0)
    nb = 3
    w = BlockWorkload(ctx, 20_000, nb, nc=25, ns=60, dirty=1_000, emit=True)
    # the oracle mirror of the state after the setup block
    n = w.n
    kk = w.keys.view(n, 32).cpu().numpy()
    vo = w.voff.cpu().numpy()
    vb = w.vals.cpu().numpy()
    ost = oracle.Trie()
    a_keys, a_vals, a_voff, cnt = w.ups[0]
    setup_bodies = {a_keys[32 * i:32 * i + 32].cpu().numpy().tobytes():
                    a_vals[int(a_voff[i]):int(a_voff[i + 1])].cpu().numpy().tobytes() for i in range(cnt)}
    for i in range(n):
        k = kk[i].tobytes()
        ost.put(k, setup_bodies.get(k, vb[vo[i]:vo[i + 1]].tobytes()))
    assert ost.root_hash() == w.state.get_root()
    s_tid, s_keys, s_vals, s_voff = w.slot_ups[0]
    ostor = {}
    tid, skb, svb, svo = (x.cpu().numpy() for x in (s_tid, s_keys, s_vals, s_voff))
    for i in range(len(tid)):
        ostor.setdefault(int(tid[i]), oracle.Trie()).put(oracle.kec256(skb[32 * i:32 * i + 32].tobytes()),
                                                        svb[svo[i]:svo[i + 1]].tobytes())
    for c in range(w.nc):
        assert ostor[c].root_hash() == w.roots[c], c
    s_store, a_store = {}, {}
    for o in ostor.values():
        s_store.update(reachable(o))
    a_store.update(reachable(ost))
    settle(list(ostor.values()) + [ost])
    for b in range(nb):
        ops = w.prepare(b)
        root = w.commit_prepared(ops)
        s_tid, s_keys, s_vals, s_voff, d_tid, d_keys, a_keys, a_vals, a_voff, a_tid, a_del = (
            None if x is None else x.cpu().numpy() for x in ops)
        for i in range(len(s_tid)):
            ostor[int(s_tid[i])].put(oracle.kec256(s_keys[32 * i:32 * i + 32].tobytes()),
                                     s_vals[s_voff[i]:s_voff[i + 1]].tobytes())
        for i in range(len(d_tid)):
            ostor[int(d_tid[i])].remove(oracle.kec256(d_keys[32 * i:32 * i + 32].tobytes()))
        touched = sorted(set(int(x) for x in s_tid) | set(int(x) for x in d_tid))
        assert sorted(w.forest.last_roots()) == touched
        for c in touched:
            assert ostor[c].root_hash() == w.roots[c], (b, c)
        fdelta = w.forest.nodes()
        check_delta(fdelta, [ostor[c] for c in touched], s_store, ("storage delta, block", b))
        s_store.update(fdelta)
        # accounts: the bodies as committed (the contracts' stateRoot fields patched)
        for i in range(len(a_tid)):
            ost.put(a_keys[32 * i:32 * i + 32].tobytes(), a_vals[a_voff[i]:a_voff[i + 1]].tobytes())
        for i in range(len(a_del) // 32):
            ost.remove(a_del[32 * i:32 * i + 32].tobytes())
        assert ost.root_hash() == root, b
        adelta = w.state.nodes()
        check_delta(adelta, [ost], a_store, ("account delta, block", b))
        a_store.update(adelta)
        settle(list(ostor.values()) + [ost])
    torch.cuda.synchronize()
