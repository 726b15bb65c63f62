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


def _host_ops(ops):
    """BlockWorkload.prepare's device tensors -> host arrays for kh_block_commit_host (the JVM's
    path: the library stages them itself)."""
    s_tid, s_keys, s_vals, s_voff, d_tid, d_keys, a_keys, a_vals, a_voff, a_tid, a_del = ops
    h = lambda t: None if t is None else t.cpu().numpy()
    na = a_tid.numel()
    return dict(s_up_trie=h(s_tid).astype(np.uint32), s_up_keys=h(s_keys), s_up_vals=h(s_vals),
                s_up_voff=h(s_voff).astype(np.uint64), s_del_trie=h(d_tid).astype(np.uint32), s_del_keys=h(d_keys),
                a_up_keys=h(a_keys), a_up_vals=h(a_vals), a_up_voff=h(a_voff)[:na + 1].astype(np.uint64),
                a_up_trie=h(a_tid).astype(np.uint32), a_del_keys=h(a_del))


def test_block_commits_on_two_host_handles_overlap(khst):
    """handles opened through the host entry points run on private contexts
    with their own locks (kh_trie::priv), so two threads committing configs[2]-shaped blocks
    (tests/blocks.py: 20k dirty accounts, 2,000 storage tries x 10 slots, storage roots injected)
    to two (state trie, forest) pairs run at once, each on its own streams.  Every root of every
    block equals the device-API reference commit of the same block (tests/test_gpu_configs.py
    checks that path against the CPU batch builder and the oracle); the two-thread throughput
    against one thread committing the same blocks to both pairs in turn is reported (0.92-1.12x
    measured: the two commits share the GPU's dispatcher)."""
    import time
    import torch
    from khipu_amd import _lib
    from khipu_amd._lib import KhStats, check, lib
    from khipu_amd.device import Ctx, block_commit_host
    from tests.blocks import BlockWorkload, hash_keys
    ctx = Ctx(0)
    n, nb = 1_000_000, 12
    w = BlockWorkload(ctx, n, nb, seed=21)
    ops = [w.prepare(b) for b in range(nb)]
    host_ops = [_host_ops(o) for o in ops]
    ref = [w.commit_prepared(tuple(x.clone() if x is not None else None for x in o)) for o in ops]
    # the initial state on the host (as the JVM holds it), the setup block's ops
    keys0 = w.keys.cpu().numpy()
    vals0 = w.vals[:int(w.voff[n])].cpu().numpy()
    voff0 = w.voff[:n + 1].cpu().numpy().astype(np.uint64)
    s_tid, s_keys, s_vals, s_voff = w.slot_ups[0]
    a_keys, a_vals, a_voff, na = w.ups[0]
    setup = dict(s_up_trie=s_tid.cpu().numpy().astype(np.uint32), s_up_keys=s_keys.cpu().numpy(),
                 s_up_vals=s_vals.cpu().numpy(), s_up_voff=s_voff.cpu().numpy().astype(np.uint64), s_del_trie=None,
                 s_del_keys=None, a_up_keys=a_keys.cpu().numpy(), a_up_vals=w.ups_pristine[0].cpu().numpy(),
                 a_up_voff=a_voff.cpu().numpy()[:na + 1].astype(np.uint64),
                 a_up_trie=np.arange(w.nc, dtype=np.uint32), a_del_keys=None)

    class H:  # a host-opened handle as block_commit_host expects it
        def __init__(self, h):
            self.h, self.ctx, self.root = h, ctx, None

    def open_pair():
        sh, fh = ctypes.c_void_p(), ctypes.c_void_p()
        root = np.zeros(32, np.uint8)
        check(lib().kh_trie_open_host(keys0.ctypes.data, 32, vals0.ctypes.data, voff0.ctypes.data, n, 0,
                                      root.ctypes.data, ctypes.byref(sh)))
        check(lib().kh_forest_open(None, _lib.KH_HASH_KEYS, ctypes.byref(fh)))
        s, f = H(sh), H(fh)
        block_commit_host(s, f, **setup)
        return s, f

    def run(pair, out, t):
        s, f = pair
        t0 = time.perf_counter()
        for o in host_ops:
            out.append(block_commit_host(s, f, **o))
        t.append(time.perf_counter() - t0)

    pairs = [open_pair() for _ in range(4)]
    # one thread: pair 0 then pair 1
    seq, tseq = [[], []], []
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    run(pairs[0], seq[0], [])
    run(pairs[1], seq[1], [])
    tseq = time.perf_counter() - t0
    # two threads: pairs 2 and 3 at once
    con, tcon = [[], []], [[], []]
    ths = [threading.Thread(target=run, args=(pairs[2 + k], con[k], tcon[k])) for k in range(2)]
    t0 = time.perf_counter()
    for t in ths:
        t.start()
    for t in ths:
        t.join(300)
    tpar = time.perf_counter() - t0
    for roots in seq + con:
        assert roots == ref, [r.hex()[:8] for r in roots]
    speedup = tseq / tpar
    print(f"two handles: one thread {tseq * 1e3 / (2 * nb):.3f} ms/block, two threads {tpar * 1e3 / (2 * nb):.3f} "
          f"ms/block, throughput x{speedup:.2f}", flush=True)
    for s, f in pairs:
        check(lib().kh_trie_free(s.h))
        check(lib().kh_trie_free(f.h))
    # Throughput is reported, not gated: measured 0.92-1.12x across boxes (scripts/concurrency_probe.py,
    # profiles/r8n_*, r8v_*: beside each other every kernel of the two commits takes 1.1-2.5x longer,
    # the dispatcher is what they share).  The floor catches a pathological slowdown of two
    # committing threads (a lock held across a sync, a shared workspace re-grown per call).
    assert speedup >= 0.75, speedup
