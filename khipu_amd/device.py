"""Device-resident interface of libkhst.so for inputs already in HBM.

torch is used only as the HBM allocator (tensors' data pointers are handed to
the C ABI); all compute is libkhst.so's HIP kernels.
"""
import ctypes

import numpy as np

from . import _lib
from ._lib import KhStats, check, lib


def _ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


class Ctx:
    """One kh_ctx (device workspace + HIP stream) per GPU."""

    def __init__(self, device=0):
        import torch
        self.torch = torch
        self.device = device
        torch.cuda.set_device(device)
        h = ctypes.c_void_p()
        check(lib().kh_ctx_create(device, ctypes.byref(h)))
        self.h = h

    def close(self):
        if self.h:
            lib().kh_ctx_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _sync(self):
        self.torch.cuda.synchronize(self.device)

    def synth_accounts(self, cfg, first, n):
        """Synthetic accounts [first, first+n) of config cfg (csrc/synth.h):
        (addresses uint8[n*20], values uint8[<=96n], offsets int64[n+1]) on the device."""
        t = self.torch
        dev = f"cuda:{self.device}"
        addr = t.empty(n * 20 + 64, dtype=t.uint8, device=dev)
        vals = t.empty(n * 96 + 64, dtype=t.uint8, device=dev)
        voff = t.empty(n + 1, dtype=t.int64, device=dev)
        self._sync()
        check(lib().kh_dev_synth_accounts(self.h, cfg, first, n, _ptr(addr), _ptr(vals), _ptr(voff)))
        return addr, vals, voff

    def storage_slot_counts(self, cfg, t0, nt):
        """Slot offsets int64[nt+1] (device) of synthetic storage tries [t0, t0+nt) and the total."""
        t = self.torch
        so = t.empty(nt + 1, dtype=t.int64, device=f"cuda:{self.device}")
        ns, vb = ctypes.c_uint64(), ctypes.c_uint64()
        self._sync()
        check(lib().kh_dev_synth_storage(self.h, cfg, t0, nt, _ptr(so), ctypes.byref(ns), ctypes.byref(vb), None, None,
                                         None, None))
        return so, int(ns.value), int(vb.value)

    def synth_storage(self, cfg, t0, nt):
        """Synthetic storage tries [t0, t0+nt) of config cfg (csrc/synth.h): (slot offsets
        int64[nt+1], keys uint8[n*32] (32-byte slot words: build with hash_keys), values,
        value offsets int64[n+1], segment ids int32[n]) on the device."""
        t = self.torch
        dev = f"cuda:{self.device}"
        so, n, vb = self.storage_slot_counts(cfg, t0, nt)
        keys = t.empty(n * 32 + 64, dtype=t.uint8, device=dev)
        vals = t.empty(vb + 64, dtype=t.uint8, device=dev)
        voff = t.empty(n + 1, dtype=t.int64, device=dev)
        seg = t.empty(n + 16, dtype=t.int32, device=dev)
        ns, vb2 = ctypes.c_uint64(), ctypes.c_uint64()
        check(lib().kh_dev_synth_storage(self.h, cfg, t0, nt, _ptr(so), ctypes.byref(ns), ctypes.byref(vb2),
                                         _ptr(keys), _ptr(vals), _ptr(voff), _ptr(seg)))
        return so, keys, vals, voff, seg

    def kec256(self, data, off, n):
        t = self.torch
        out = t.empty(32 * max(n, 1), dtype=t.uint8, device=data.device)
        self._sync()
        check(lib().kh_dev_kec256_batch(self.h, _ptr(data), _ptr(off), n, _ptr(out)))
        self._sync()
        return out[:32 * n]

    def build(self, keys, klen, vals, voff, n, seg=None, nseg=1, depth0=0, hash_keys=False, vals_ready=None):
        """Returns (hash32 [nres,32] uint8, enc_len [nres] uint32, inline [nres,32] uint8, KhStats).
        vals_ready: a torch.cuda.Event after which vals / voff are in place
        (kh_dev_trie_build_ev); the keys must be in place already, and the build does
        not synchronise the device first."""
        nres = nseg if seg is not None else (16 if depth0 == 1 else 1)
        hh = np.zeros(32 * nres, np.uint8)
        ll = np.zeros(nres, np.uint32)
        ii = np.zeros(32 * nres, np.uint8)
        st = KhStats()
        flags = _lib.KH_HASH_KEYS if hash_keys else 0
        if vals_ready is None:
            self._sync()
            ev = None
        else:
            ev = ctypes.c_void_p(vals_ready.cuda_event)
        check(lib().kh_dev_trie_build_ev(self.h, ev, _ptr(keys), klen, _ptr(vals), _ptr(voff), n, _ptr(seg), nseg,
                                         depth0, flags, hh.ctypes.data, ll.ctypes.data, ii.ctypes.data,
                                         ctypes.byref(st)))
        return hh.reshape(nres, 32), ll, ii.reshape(nres, 32), st

    def list_roots(self, items, off, seg_off):
        """kh_dev_list_roots: items / off (n + 1 int64 offsets) device tensors, seg_off host
        (numpy uint64, nseg + 1).  Returns (list of 32-byte roots, KhStats)."""
        so = np.ascontiguousarray(seg_off, dtype=np.uint64)
        nseg = len(so) - 1
        out = np.zeros(32 * max(nseg, 1), np.uint8)
        st = KhStats()
        self._sync()
        check(lib().kh_dev_list_roots(self.h, _ptr(items), _ptr(off), so.ctypes.data, nseg, out.ctypes.data,
                                      ctypes.byref(st)))
        return [out[32 * i:32 * i + 32].tobytes() for i in range(nseg)], st


def fold_root16(hash32x16, len16, inline32x16):
    """Root over 16 capped top-nibble references (kh_fold_root16)."""
    hh = np.ascontiguousarray(hash32x16, dtype=np.uint8).reshape(-1)
    ll = np.ascontiguousarray(len16, dtype=np.uint32)
    ii = np.ascontiguousarray(inline32x16, dtype=np.uint8).reshape(-1)
    out = np.zeros(32, np.uint8)
    check(lib().kh_fold_root16(hh.ctypes.data, ll.ctypes.data, ii.ctypes.data, out.ctypes.data))
    return out.tobytes()


def _pack_dev(items, device):
    """bytes list -> (uint8 data, int64 offsets[n+1]) tensors on the device."""
    import torch
    blob = b"".join(items)
    data = torch.zeros(len(blob) + 64, dtype=torch.uint8)
    if blob:
        data[:len(blob)] = torch.frombuffer(bytearray(blob), dtype=torch.uint8)
    off = torch.tensor(np.concatenate([[0], np.cumsum([len(x) for x in items], dtype=np.int64)]).astype(np.int64))
    return data.to(device), off.to(device)


class _Versioned:
    """Versioned commits shared by ResidentTrie and ResidentForest (kh_trie_savepoint /
    kh_trie_rollback / kh_trie_release; Ledger.executeBlock's retry from the parent state,
    Ledger.scala:237-271, and the rejection of validateBlockAfterExecution, :603-620)."""

    def savepoint(self):
        """Open a savepoint (they nest); returns the number now open."""
        d = ctypes.c_uint32()
        check(lib().kh_trie_savepoint(self.h, ctypes.byref(d)))
        return int(d.value)

    def rollback(self):
        """Back to the innermost savepoint's version (root, records, last roots, write-back set)."""
        self.ctx._sync()
        check(lib().kh_trie_rollback(self.h))
        self._after_rollback()

    def release(self):
        """Keep the commits since the innermost savepoint and close it."""
        check(lib().kh_trie_release(self.h))

    def savepoint_depth(self):
        d = ctypes.c_uint32()
        check(lib().kh_trie_savepoint_depth(self.h, ctypes.byref(d)))
        return int(d.value)

    def _after_rollback(self):
        pass

    def usage(self):
        """{records, live_records, heap_bytes, live_heap_bytes, map_slots, hbm_bytes} (kh_trie_usage)."""
        u = _lib.KhTrieUsage()
        self.ctx._sync()
        check(lib().kh_trie_usage(self.h, ctypes.byref(u)))
        return {f: int(getattr(u, f)) for f, _ in u._fields_}

    def compact(self):
        """Rewrite the live records and values densely (kh_trie_compact); the version is unchanged.
        Returns {records, heap_bytes} before it."""
        u = _lib.KhTrieUsage()
        self.ctx._sync()
        check(lib().kh_trie_compact(self.h, ctypes.byref(u)))
        return {"records": int(u.records), "heap_bytes": int(u.heap_bytes)}


class ResidentTrie(_Versioned):
    """A trie kept in HBM between commits (kh_trie_open / kh_trie_apply).

    commit(upserts, deletes) folds a block's dirty set the way TrieAccounts.flush /
    TrieStorage.flush fold their logs into MerklePatriciaTrie.put / remove
    (TrieAccounts.scala:22-28, TrieStorage.scala:43-60), rebuilding only the nodes on the
    changed paths (csrc/forest.h).  Keys are 32-byte trie keys, or raw (address / slot)
    bytes with hash_keys.  With emit=True, nodes() returns the write-back set of the last
    commit (the nodes it created).
    """

    def __init__(self, ctx, keys=(), vals=(), hash_keys=False, emit=True):
        self.ctx = ctx
        self.dev = f"cuda:{ctx.device}"
        self.h = None
        klen = len(keys[0]) if keys else 32
        kd, _ = _pack_dev(list(keys), self.dev)
        vd, vo = _pack_dev(list(vals), self.dev)
        self._open(kd, klen, vd, vo, len(keys), hash_keys, emit)

    def _open(self, kd, klen, vd, vo, n, hash_keys, emit=True):
        self.hash_keys = bool(hash_keys)  # every commit hashes its keys the same way
        h = ctypes.c_void_p()
        root = np.zeros(32, np.uint8)
        flags = (_lib.KH_HASH_KEYS if hash_keys else 0) | (_lib.KH_EMIT_NODES if emit else 0)
        self.ctx._sync()
        check(lib().kh_trie_open(self.ctx.h, _ptr(kd), klen, _ptr(vd), _ptr(vo), n, flags, root.ctypes.data,
                                 ctypes.byref(h)))
        self.h = h
        self.root = root.tobytes()

    @classmethod
    def from_nodes(cls, ctx, root, nodes, hash_keys=False, emit=True):
        """Open from a root hash and a node store {hash: encoding} (kh_trie_open_nodes;
        MerklePatriciaTrie.apply(rootHash, source)).  A missing node raises
        MPTNodeMissingException with the missing hash in .missing."""
        t = cls.__new__(cls)
        t.ctx, t.dev, t.h = ctx, f"cuda:{ctx.device}", None
        t.hash_keys = bool(hash_keys)
        encs = list(nodes.values())
        ed, eo = _pack_dev(encs, t.dev)
        h = ctypes.c_void_p()
        miss = np.zeros(32, np.uint8)
        flags = (_lib.KH_HASH_KEYS if hash_keys else 0) | (_lib.KH_EMIT_NODES if emit else 0)
        rb = np.frombuffer(bytes(root), np.uint8).copy()
        ctx._sync()
        rc = lib().kh_trie_open_nodes(ctx.h, rb.ctypes.data, _ptr(ed), _ptr(eo), len(encs), flags, miss.ctypes.data,
                                      ctypes.byref(h))
        if rc == _lib.KH_ENODE:
            e = _lib.MPTNodeMissingException(rc, lib().kh_last_error().decode())
            e.missing = miss.tobytes()
            raise e
        check(rc)
        t.h = h
        t.root = bytes(root)
        return t

    def _flag(self, hash_keys):
        """The trie's key encoder is fixed at open (as the reference's implicit
        ByteArrayEncoder[K] is per trie type): None means that one; a different value raises."""
        if hash_keys is None:
            return self.hash_keys
        if bool(hash_keys) != self.hash_keys:
            raise _lib.MPTException(_lib.KH_EINVAL, f"trie opened with hash_keys={self.hash_keys}, commit asked "
                                                    f"for hash_keys={bool(hash_keys)}")
        return self.hash_keys

    def commit(self, upserts=(), deletes=(), hash_keys=None, stats=None):
        """Apply {key: value} upserts, then deletes; returns the new root."""
        ups = list(upserts.items()) if isinstance(upserts, dict) else list(upserts)
        dels = list(deletes)
        klen = len(ups[0][0]) if ups else (len(dels[0]) if dels else 32)
        uk, _ = _pack_dev([k for k, _ in ups], self.dev)
        uv, uo = _pack_dev([v for _, v in ups], self.dev)
        dk, _ = _pack_dev(dels, self.dev)
        return self.commit_dev(uk, uv, uo, len(ups), dk, len(dels), klen, hash_keys, stats)

    def commit_dev(self, up_keys, up_vals, up_voff, nup, del_keys, ndel, klen=32, hash_keys=None, stats=None):
        root = np.zeros(32, np.uint8)
        st = stats if stats is not None else KhStats()
        flags = _lib.KH_HASH_KEYS if self._flag(hash_keys) else 0
        self.ctx._sync()
        check(lib().kh_trie_apply(self.h, _ptr(up_keys), _ptr(up_vals), _ptr(up_voff), nup, _ptr(del_keys), ndel,
                                  klen, flags, root.ctypes.data, ctypes.byref(st)))
        self.root = root.tobytes()
        return self.root

    def nodes(self):
        """{hash: encoding} written back by the last commit (kh_trie_emit_nodes): the nodes it
        created, every one reachable from the new root with an encoding >= 32 B, plus a changed root."""
        return emitted_nodes(lambda *a: lib().kh_trie_emit_nodes(self.h, *a))

    def root_of(self, upserts=(), deletes=(), stats=None):
        """TrieAccounts.rootHash (TrieAccounts.scala:73-80): the root commit(upserts, deletes)
        would give; the trie is left unchanged (kh_trie_root_of)."""
        ups = list(upserts.items()) if isinstance(upserts, dict) else list(upserts)
        dels = list(deletes)
        klen = len(ups[0][0]) if ups else (len(dels[0]) if dels else 32)
        uk, _ = _pack_dev([k for k, _ in ups], self.dev)
        uv, uo = _pack_dev([v for _, v in ups], self.dev)
        dk, _ = _pack_dev(dels, self.dev)
        root = np.zeros(32, np.uint8)
        st = stats if stats is not None else KhStats()
        flags = _lib.KH_HASH_KEYS if self.hash_keys else 0
        self.ctx._sync()
        check(lib().kh_trie_root_of(self.h, _ptr(uk), _ptr(uv), _ptr(uo), len(ups), _ptr(dk), len(dels), klen, flags,
                                    root.ctypes.data, ctypes.byref(st)))
        return root.tobytes()

    def copy(self):
        """MerklePatriciaTrie.copy (MerklePatriciaTrie.scala:556): an independent resident trie
        holding the current version (kh_trie_copy)."""
        h = ctypes.c_void_p()
        self.ctx._sync()
        check(lib().kh_trie_copy(self.h, ctypes.byref(h)))
        t = ResidentTrie.__new__(ResidentTrie)
        t.ctx, t.dev, t.h, t.hash_keys, t.root = self.ctx, self.dev, h, self.hash_keys, self.root
        return t

    def _after_rollback(self):
        self.root = self.get_root()

    def get_root(self):
        """The handle's current root (kh_trie_root_of of an empty batch)."""
        root = np.zeros(32, np.uint8)
        check(lib().kh_trie_root_of(self.h, None, None, None, 0, None, 0, 32,
                                    _lib.KH_HASH_KEYS if self.hash_keys else 0, root.ctypes.data, None))
        return root.tobytes()

    def get(self, keys):
        """Batched get (kh_trie_get): [value or None] per key (raw keys with hash_keys)."""
        return trie_get(self.h, keys)

    @property
    def root_hash(self):
        return self.root

    def __len__(self):
        n = ctypes.c_uint64()
        check(lib().kh_trie_size(self.h, ctypes.byref(n)))
        return int(n.value)

    def close(self):
        if self.h:
            lib().kh_trie_free(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def trie_get(h, keys, trie_ids=None):
    """Batched get through kh_trie_get_host: [value bytes or None] per key
    (MerklePatriciaTrie.get, MerklePatriciaTrie.scala:90-147)."""
    keys = list(keys)
    n = len(keys)
    klen = len(keys[0]) if keys else 32
    kb = np.frombuffer(b"".join(keys) + b"\0", np.uint8).copy()
    tb = np.asarray(trie_ids, np.uint32) if trie_ids is not None else None
    found = np.zeros(max(n, 1), np.uint8)
    voff = np.zeros(n + 1, np.uint64)
    need = ctypes.c_uint64(0)
    cap = 0
    for _ in range(2):
        vals = np.zeros(max(cap, 1), np.uint8)
        rc = lib().kh_trie_get_host(h, tb.ctypes.data if tb is not None else None, kb.ctypes.data, klen, n,
                                    vals.ctypes.data, cap, voff.ctypes.data, found.ctypes.data, ctypes.byref(need))
        if rc == _lib.KH_ENOSPC:
            cap = need.value
            continue
        check(rc)
        return [vals[voff[i]:voff[i + 1]].tobytes() if found[i] else None for i in range(n)]
    raise RuntimeError("kh_trie_get: size negotiation failed")


def emitted_nodes(call):
    """Size negotiation of kh_trie_emit_nodes (KH_ENOSPC reports the sizes; no re-encoding).
    Another thread's commit on the handle may replace the set between the size query and the
    read (the reader then sees KH_ENOSPC with the new sizes): the query is repeated."""
    nn, nl = ctypes.c_uint64(0), ctypes.c_uint64(0)
    cap_n, cap_b = 0, 0
    for _ in range(16):
        hs = np.zeros(32 * max(cap_n, 1), np.uint8)
        rl = np.zeros(max(cap_b, 1), np.uint8)
        of = np.zeros(cap_n + 1, np.uint64)
        rc = call(hs.ctypes.data, cap_n, rl.ctypes.data, cap_b, of.ctypes.data, ctypes.byref(nn), ctypes.byref(nl))
        if rc == _lib.KH_ENOSPC:
            cap_n, cap_b = nn.value, nl.value
            continue
        check(rc)
        return {hs[32 * i:32 * i + 32].tobytes(): rl[of[i]:of[i + 1]].tobytes() for i in range(nn.value)}
    raise RuntimeError("kh_trie_emit_nodes: size negotiation failed")


class ResidentForest(_Versioned):
    """Many tries in one handle (contract storage tries; kh_forest_open / kh_forest_apply,
    SURVEY §8 a12): each op names its trie id; one commit re-roots every touched trie."""

    def __init__(self, ctx, hash_keys=False, emit=False):
        self.ctx = ctx
        self.dev = f"cuda:{ctx.device}"
        self.hash_keys = bool(hash_keys)
        h = ctypes.c_void_p()
        flags = (_lib.KH_HASH_KEYS if hash_keys else 0) | (_lib.KH_EMIT_NODES if emit else 0)
        check(lib().kh_forest_open(ctx.h, flags, ctypes.byref(h)))
        self.h = h

    def commit(self, upserts=(), deletes=(), stats=None):
        """upserts: [(trie_id, key, value)], deletes: [(trie_id, key)] -> {trie_id: new root}."""
        import torch
        ups, dels = list(upserts), list(deletes)
        klen = len(ups[0][1]) if ups else (len(dels[0][1]) if dels else 32)
        uk, _ = _pack_dev([k for _, k, _ in ups], self.dev)
        uv, uo = _pack_dev([v for _, _, v in ups], self.dev)
        dk, _ = _pack_dev([k for _, k in dels], self.dev)
        ut = torch.tensor([t for t, _, _ in ups] + [0], dtype=torch.int64).to(torch.int32).to(self.dev)
        dt = torch.tensor([t for t, _ in dels] + [0], dtype=torch.int64).to(torch.int32).to(self.dev)
        cap = len(ups) + len(dels) + 1
        tries = np.zeros(cap, np.uint32)
        roots = np.zeros(32 * cap, np.uint8)
        nt = ctypes.c_uint64()
        st = stats if stats is not None else KhStats()
        self.ctx._sync()
        check(lib().kh_forest_apply(self.h, _ptr(ut), _ptr(uk), _ptr(uv), _ptr(uo), len(ups), _ptr(dt), _ptr(dk),
                                    len(dels), klen, tries.ctypes.data, roots.ctypes.data, cap, ctypes.byref(nt),
                                    ctypes.byref(st)))
        return {int(tries[i]): roots[32 * i:32 * i + 32].tobytes() for i in range(nt.value)}

    def nodes(self):
        return emitted_nodes(lambda *a: lib().kh_trie_emit_nodes(self.h, *a))

    def get(self, queries):
        """queries: [(trie_id, key)] -> [value or None] (kh_trie_get)."""
        q = list(queries)
        return trie_get(self.h, [k for _, k in q], [t for t, _ in q])

    def last_roots(self):
        """{trie_id: root} of the last commit (kh_forest_last_roots; also after block_commit)."""
        n = ctypes.c_uint64()
        rc = lib().kh_forest_last_roots(self.h, None, None, 0, ctypes.byref(n))
        if rc not in (_lib.KH_OK, _lib.KH_ENOSPC):
            check(rc)
        cap = n.value
        tries = np.zeros(max(cap, 1), np.uint32)
        roots = np.zeros(32 * max(cap, 1), np.uint8)
        check(lib().kh_forest_last_roots(self.h, tries.ctypes.data, roots.ctypes.data, cap, ctypes.byref(n)))
        return {int(tries[i]): roots[32 * i:32 * i + 32].tobytes() for i in range(n.value)}

    def __len__(self):
        n = ctypes.c_uint64()
        check(lib().kh_trie_size(self.h, ctypes.byref(n)))
        return int(n.value)

    def close(self):
        if self.h:
            lib().kh_trie_free(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def block_commit(state, forest, s_up_trie, s_up_keys, s_up_vals, s_up_voff, ns_up, s_del_trie, s_del_keys, ns_del,
                 a_up_keys, a_up_vals, a_up_voff, a_up_trie, na_up, a_del_keys, na_del, s_klen=32, a_klen=32,
                 stats=None):
    """One block through kh_block_commit (device tensors): the storage ops into the forest,
    the touched tries' new roots written into the stateRoot of the account upserts that name
    them (a_up_trie, KH_NO_TRIE for none; a_up_vals is patched in place), then the account
    ops into the state trie.  Returns the new state root."""
    root = np.zeros(32, np.uint8)
    st = stats if stats is not None else KhStats()
    state.ctx._sync()
    check(lib().kh_block_commit(state.h, forest.h, _ptr(s_up_trie), _ptr(s_up_keys), _ptr(s_up_vals), _ptr(s_up_voff),
                                ns_up, _ptr(s_del_trie), _ptr(s_del_keys), ns_del, s_klen, _ptr(a_up_keys),
                                _ptr(a_up_vals), _ptr(a_up_voff), _ptr(a_up_trie), na_up, _ptr(a_del_keys), na_del,
                                a_klen, root.ctypes.data, ctypes.byref(st)))
    state.root = root.tobytes()
    return state.root


def block_commit_host(state, forest, s_up_trie, s_up_keys, s_up_vals, s_up_voff, s_del_trie, s_del_keys,
                      a_up_keys, a_up_vals, a_up_voff, a_up_trie, a_del_keys, s_klen=32, a_klen=32, stats=None):
    """kh_block_commit_host: the same block from host (numpy) arrays; counts from the shapes."""
    keep = []  # contiguous copies stay alive through the call

    def p(a):
        if a is None:
            return None
        a = np.ascontiguousarray(a)
        keep.append(a)
        return a.ctypes.data
    ns_up = 0 if s_up_trie is None else len(s_up_trie)
    ns_del = 0 if s_del_trie is None else len(s_del_trie)
    na_up = len(a_up_voff) - 1
    na_del = 0 if a_del_keys is None else len(a_del_keys) // a_klen
    root = np.zeros(32, np.uint8)
    st = stats if stats is not None else KhStats()
    state.ctx._sync()
    check(lib().kh_block_commit_host(state.h, forest.h, p(s_up_trie), p(s_up_keys), p(s_up_vals), p(s_up_voff), ns_up,
                                     p(s_del_trie), p(s_del_keys), ns_del, s_klen, p(a_up_keys), p(a_up_vals),
                                     p(a_up_voff), p(a_up_trie), na_up, p(a_del_keys), na_del, a_klen,
                                     root.ctypes.data, ctypes.byref(st)))
    del keep
    state.root = root.tobytes()
    return state.root
