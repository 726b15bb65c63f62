"""The boundary's threading contract (include/khst.h "Threading"): host entry points called
from several JVM threads at once on handles of the shared context.  The reference drives
the trie from many worker threads (TxProcessor.scala:28-35 runs up to 1,000), each block's
world state on its own trie; BlockWorldState.persist hands each one's write-back set to the
node store (BlockWorldState.scala:312-330).

Two threads each commit blocks to their own host-opened trie (kh_trie_open_host /
kh_trie_apply_host, both on the shared context) and read their write-back set right after
each commit (kh_trie_emit_nodes); a third thread keeps reading both handles' write-back sets,
usage, size and savepoint depth, and opens / releases savepoints on them.  Every root equals
the oracle's fold, every delta satisfies the strict f2 contract (tests/writeback.py), and
every set the reader saw is one that a commit produced."""
import ctypes
import random
import threading

import numpy as np
import pytest

from tests import cases as C
from tests.writeback import check_delta, reachable, settle

pytestmark = pytest.mark.gpu

BLOCKS = 10


def _pack(items):
    b = np.frombuffer(b"".join(items) + bytes(16), np.uint8)
    off = np.concatenate([[0], np.cumsum([len(x) for x in items])]).astype(np.uint64)
    return b, off


def _open(lib, check, _lib, keys, vals):
    kb, _ = _pack(keys)
    vb, vo = _pack(vals)
    h = ctypes.c_void_p()
    root = np.zeros(32, np.uint8)
    check(lib().kh_trie_open_host(kb.ctypes.data, 32, vb.ctypes.data, vo.ctypes.data, len(keys), _lib.KH_EMIT_NODES,
                                  root.ctypes.data, ctypes.byref(h)))
    return h, root.tobytes()


def test_two_committers_and_a_reader_on_the_shared_context(khst, oracle):
    from khipu_amd import _lib
    from khipu_amd._lib import check, lib
    from khipu_amd.device import emitted_nodes
    handles, oracles, seen_by_committer = [], [], [[], []]
    for w in range(2):
        r = random.Random(100 + w)
        keys = [bytes(r.getrandbits(8) for _ in range(32)) for _ in range(3000)]
        vals = [C.account_value(r) for _ in keys]
        o = oracle.Trie()
        for k, v in zip(keys, vals):
            o.put(k, v)
        h, root = _open(lib, check, _lib, keys, vals)
        assert root == o.root_hash()
        settle([o])
        handles.append((h, keys))
        oracles.append(o)
    errors = []
    stop = threading.Event()

    def committer(w):
        try:
            h, keys = handles[w]
            o = oracles[w]
            store = dict(reachable(o))
            r = random.Random(200 + w)
            live = list(keys)
            for blk in range(BLOCKS):
                ups = [(k, C.account_value(r)) for k in r.sample(live, 150)]
                ups += [(bytes(r.getrandbits(8) for _ in range(32)), C.account_value(r)) for _ in range(40)]
                dels = r.sample(live, 20)
                uk, _ = _pack([k for k, _ in ups])
                uv, uo = _pack([v for _, v in ups])
                dk, _ = _pack(dels)
                root = np.zeros(32, np.uint8)
                check(lib().kh_trie_apply_host(h, uk.ctypes.data, uv.ctypes.data, uo.ctypes.data, len(ups),
                                               dk.ctypes.data, len(dels), 32, 0, root.ctypes.data, None))
                delta = emitted_nodes(lambda *a: lib().kh_trie_emit_nodes(h, *a))
                for k, v in ups:
                    o.put(k, v)
                for k in dels:
                    o.remove(k)
                assert root.tobytes() == o.root_hash(), (w, blk)
                store.update(check_delta(delta, [o], store, f"thread {w} block {blk}"))
                settle([o])
                seen_by_committer[w].append(frozenset(delta))
                live = [k for k in live if k not in set(dels)] + [k for k, _ in ups[150:]]
        except BaseException as e:  # reported by the main thread
            errors.append(("committer", w, repr(e)))

    seen_by_reader = [set(), set()]
    reads = [0]

    def reader():
        try:
            u = _lib.KhTrieUsage()
            n = ctypes.c_uint64()
            d = ctypes.c_uint32()
            it = 0
            while not stop.is_set():
                w = it & 1
                h = handles[w][0]
                seen_by_reader[w].add(frozenset(emitted_nodes(lambda *a: lib().kh_trie_emit_nodes(h, *a))))
                check(lib().kh_trie_usage(h, ctypes.byref(u)))
                check(lib().kh_trie_size(h, ctypes.byref(n)))
                if it % 7 == 3:  # a savepoint opened and released between the other threads' commits
                    check(lib().kh_trie_savepoint(h, ctypes.byref(d)))
                    check(lib().kh_trie_savepoint_depth(h, ctypes.byref(d)))
                    assert d.value >= 1
                    check(lib().kh_trie_release(h))
                it += 1
                reads[0] = it
        except BaseException as e:
            errors.append(("reader", repr(e)))

    ts = [threading.Thread(target=committer, args=(w,)) for w in range(2)]
    tr = threading.Thread(target=reader)
    tr.start()
    for t in ts:
        t.start()
    for t in ts:
        t.join(300)
    stop.set()
    tr.join(60)
    assert not errors, errors
    assert all(len(s) == BLOCKS for s in seen_by_committer)
    assert reads[0] > 10
    for w in range(2):
        # the reader saw the open's set (before the first commit) or a set some commit produced
        extra = seen_by_reader[w] - set(seen_by_committer[w])
        assert len(extra) <= 1, (w, len(extra))
    for h, _ in handles:
        check(lib().kh_trie_free(h))
