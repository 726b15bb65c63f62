"""GPU tests of resident-trie compaction (kh_trie_compact / kh_trie_usage): the records and
value heap of a resident trie or forest grow with every commit (replaced records stay behind,
dead); a compaction rewrites the live ones densely and must leave the version untouched --
root, get() answers, size, write-back set and last roots -- while later commits keep matching
the khipu-faithful oracle's fold (MerklePatriciaTrie.put / remove, MerklePatriciaTrie.scala:157-477)."""
import random

import pytest

from tests import cases as C

pytestmark = pytest.mark.gpu


def _oracle(oracle, ks, vs):
    o = oracle.Trie()
    for k, v in zip(ks, vs):
        o.put(k, v)
    return o


def test_compact_trie_keeps_version_and_later_commits(khst, oracle):
    from khipu_amd.device import Ctx, ResidentTrie
    r = random.Random(31)
    ks = [C._rk(r) for _ in range(20_000)]
    vs = [C.account_value(r) for _ in ks]
    t = ResidentTrie(Ctx(0), ks, vs)
    o = _oracle(oracle, ks, vs)
    live = dict(zip(ks, vs))
    for b in range(6):  # updates, inserts, removes: dead records and values pile up
        ups = [(k, C.account_value(r)) for k in r.sample(sorted(live), 1500)] + \
              [(C._rk(r), C.account_value(r)) for _ in range(500)]
        dels = r.sample(sorted(live), 300)
        for k, v in ups:
            o.put(k, v)
            live[k] = v
        for k in dels:
            o.remove(k)
            live.pop(k, None)
        assert t.commit(ups, dels) == o.root_hash(), b
    u0 = t.usage()
    assert u0["live_records"] < u0["records"] and u0["live_heap_bytes"] < u0["heap_bytes"], u0
    root, nodes, size = t.root, t.nodes(), len(t)
    probe = r.sample(sorted(live), 500) + [C._rk(r) for _ in range(50)] + dels[:50]
    got = t.get(probe)
    before = t.compact()
    assert before["records"] == u0["records"] and before["heap_bytes"] == u0["heap_bytes"]
    u1 = t.usage()
    assert u1["records"] == u1["live_records"] == u0["live_records"], (u0, u1)
    assert u1["heap_bytes"] == u1["live_heap_bytes"] == u0["live_heap_bytes"], (u0, u1)
    assert t.get_root() == root and t.nodes() == nodes and len(t) == size
    assert t.get(probe) == got == [live.get(k) for k in probe]
    for b in range(3):  # later commits (and a rollback) on the compacted records
        ups = [(k, C.account_value(r)) for k in r.sample(sorted(live), 800)] + \
              [(C._rk(r), C.account_value(r)) for _ in range(200)]
        dels = r.sample(sorted(live), 100)
        t.savepoint()
        t.commit([(k, b"\x01") for k, _ in ups[:10]], dels[:5])
        t.rollback()
        for k, v in ups:
            o.put(k, v)
            live[k] = v
        for k in dels:
            o.remove(k)
            live.pop(k, None)
        assert t.commit(ups, dels) == o.root_hash(), b
    assert t.get(probe) == [live.get(k) for k in probe]
    t.close()


def test_compact_refused_with_open_savepoint(khst, oracle):
    from khipu_amd import _lib
    from khipu_amd.device import Ctx, ResidentTrie
    r = random.Random(3)
    ks = [C._rk(r) for _ in range(300)]
    vs = [C.account_value(r) for _ in ks]
    t = ResidentTrie(Ctx(0), ks, vs)
    t.savepoint()
    t.commit([(ks[0], b"\x05")], [ks[1]])
    with pytest.raises(_lib.KhError):
        t.compact()
    t.rollback()
    t.compact()
    assert t.root == _oracle(oracle, ks, vs).root_hash() == t.get_root()
    t.close()


def test_emit_after_delete_only_commit_and_compaction(khst, oracle):
    """A commit that changes nothing (deletes of absent keys) leaves an empty write-back set;
    compaction may release its buffer, and reading the set afterwards gives 0 nodes (not a
    device error from a copy out of a released buffer)."""
    from khipu_amd.device import Ctx, ResidentTrie
    r = random.Random(4)
    ks = [C._rk(r) for _ in range(400)]
    vs = [C.account_value(r) for _ in ks]
    t = ResidentTrie(Ctx(0), ks, vs)
    root = t.root
    assert t.commit([], [C._rk(r) for _ in range(3)]) == root
    assert t.nodes() == {}
    t.compact()
    assert t.nodes() == {}
    assert t.get_root() == root == _oracle(oracle, ks, vs).root_hash()
    t.close()


def test_compact_forest(khst, oracle):
    """A storage forest: roots of every trie, last roots and get() unchanged; a later commit
    across tries equals the oracle per trie."""
    from khipu_amd.device import Ctx, ResidentForest
    r = random.Random(8)
    f = ResidentForest(Ctx(0))
    tries = {}
    for b in range(5):
        ups, dels = [], []
        for tid in r.sample(range(40), 12):
            d = tries.setdefault(tid, {})
            for _ in range(r.randint(1, 60)):
                k = C._rk(r)
                v = bytes([r.randrange(1, 256)]) * r.choice([1, 3, 33])
                d[k] = v
                ups.append((tid, k, v))
            for k in r.sample(sorted(d), min(len(d), r.randint(0, 5))):
                if all(k != kk or t != tid for t, kk, _ in ups):
                    del d[k]
                    dels.append((tid, k))
        f.commit(ups, dels)
    last = f.last_roots()
    queries = [(tid, k) for tid, d in tries.items() for k in list(d)[:20]] + [(77, C._rk(r))]
    got = f.get(queries)
    u0 = f.usage()
    f.compact()
    u1 = f.usage()
    assert u1["records"] == u0["live_records"] < u0["records"]
    assert f.last_roots() == last and f.get(queries) == got
    ups = []
    for tid in list(tries)[:10]:
        k = C._rk(r)
        tries[tid][k] = b"\x42" * 40
        ups.append((tid, k, b"\x42" * 40))
    roots = f.commit(ups, [])
    for tid in list(tries)[:10]:
        d = tries[tid]
        assert roots[tid] == oracle.seq_root(list(d), list(d.values())), tid
    f.close()
