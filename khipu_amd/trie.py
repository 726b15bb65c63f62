"""Host-side mirror of khipu's trie / crypto entry points over libkhst.so.

Mirrors the operator surface the reference exposes on the state-root path, with
the same names, argument meaning and error behaviour, but every root, node hash
and node encoding is computed by the HIP kernels of libkhst.so:

* ``kec256`` / ``kec256_batch``  — crypto.kec256 (crypto/package.scala:37-47)
* ``MerklePatriciaTrie``        — khipu.trie.MerklePatriciaTrie
  (trie/MerklePatriciaTrie.scala:57-558): put / remove / get / root_hash /
  persist / changes / copy.  ``update`` raises like the reference (:487-489).
* ``trie_root`` / ``trie_roots``  — the batch commit that TrieAccounts.flush /
  TrieStorage.flush perform (ledger/TrieAccounts.scala:22-28,
  ledger/TrieStorage.scala:52-60) as one device call.
* ``trie_roots_varkeys`` — tries over unhashed keys of any length <= 32 B (branch values).
* ``list_roots`` / ``MptListValidator`` — transactions / receipts roots over rlp(i) keys
  (validators/MptListValidator.scala:15-46, mining/BlockGenerator.scala:157-163).

The mirror keeps the trie's leaf set (key -> value bytes) on the host and
rebuilds the root on the device when it is asked for; the resulting root and
node set are the canonical ones the sequential reference reaches.
"""
import ctypes

import numpy as np

from . import _lib
from ._lib import KhStats, check, lib, MPTException

EMPTY_TRIE_HASH = bytes.fromhex("56e81f171bcc55a6ff8345e692c0f86e5b48e01b996cadc001622fb5e363b421")


def _u8(b):
    if isinstance(b, np.ndarray):
        return np.ascontiguousarray(b, dtype=np.uint8)
    return np.frombuffer(bytes(b) + b"\0" * 8, dtype=np.uint8)


def _pack(items):
    off = np.zeros(len(items) + 1, dtype=np.uint64)
    if items:
        off[1:] = np.cumsum([len(v) for v in items], dtype=np.uint64)
    return _u8(b"".join(items)), off


def kec256_batch(msgs):
    """[kec256(m) for m in msgs] in one device call."""
    n = len(msgs)
    if n == 0:
        return []
    data, off = _pack(list(msgs))
    out = np.zeros(32 * n, dtype=np.uint8)
    check(lib().kh_kec256_batch(data.ctypes.data, off.ctypes.data, n, out.ctypes.data))
    return [out[32 * i:32 * i + 32].tobytes() for i in range(n)]


def kec256(*parts) -> bytes:
    """crypto.kec256(Array[Byte]*): hash of the concatenation (crypto/package.scala:43-47)."""
    return kec256_batch([b"".join(parts)])[0]


def _keys_buf(keys, klen):
    if isinstance(keys, np.ndarray):
        kb = np.ascontiguousarray(keys, dtype=np.uint8).reshape(-1)
        n = kb.size // klen
    else:
        keys = list(keys)
        n = len(keys)
        for k in keys:
            if len(k) != klen:
                raise MPTException(_lib.KH_EINVAL, "all keys must have the same length")
        kb = _u8(b"".join(keys))
    return kb, n


def trie_root(keys, vals, hash_keys=False, klen=None, stats=None):
    """Root of the trie holding put(keys[i], vals[i]) in order (later puts win).

    keys: list of bytes (32 B, or any fixed length with hash_keys=True) or a
    uint8 array of n*klen; vals: list of bytes, or (values uint8 array, offsets
    uint64[n+1]).
    """
    if klen is None:
        klen = 32 if isinstance(keys, np.ndarray) or not keys else len(keys[0])
    kb, n = _keys_buf(keys, klen)
    vb, off = vals if isinstance(vals, tuple) else _pack(list(vals))
    vb = _u8(vb)
    out = np.zeros(32, dtype=np.uint8)
    st = stats if stats is not None else KhStats()
    flags = _lib.KH_HASH_KEYS if hash_keys else 0
    check(lib().kh_trie_root(kb.ctypes.data, klen, vb.ctypes.data, np.ascontiguousarray(off, np.uint64).ctypes.data,
                             n, flags, out.ctypes.data, ctypes.byref(st)))
    return out.tobytes()


def trie_root_sharded(keys, vals, devices, hash_keys=False, klen=None, stats=None, rccl=False):
    """trie_root on several GPUs of this process (kh_trie_root_sharded: nibble shards,
    RCCL point-to-point exchange, host fold of the 16 subtrie references).  rccl=True
    (KH_SHARD_RCCL) takes the RCCL exchange even when `devices` repeats a device, which needs
    a communicator that accepts repeats (tests/loopback)."""
    if klen is None:
        klen = 32 if isinstance(keys, np.ndarray) or not keys else len(keys[0])
    kb, n = _keys_buf(keys, klen)
    vb, off = vals if isinstance(vals, tuple) else _pack(list(vals))
    vb = _u8(vb)
    dv = np.asarray(list(devices), dtype=np.int32)
    out = np.zeros(32, dtype=np.uint8)
    st = stats if stats is not None else KhStats()
    flags = (_lib.KH_HASH_KEYS if hash_keys else 0) | (_lib.KH_SHARD_RCCL if rccl else 0)
    check(lib().kh_trie_root_sharded(dv.ctypes.data, len(dv), kb.ctypes.data, klen, vb.ctypes.data,
                                     np.ascontiguousarray(off, np.uint64).ctypes.data, n, flags, out.ctypes.data,
                                     ctypes.byref(st)))
    return out.tobytes()


def trie_roots(tries, hash_keys=False, stats=None, devices=None):
    """Roots of many independent tries in one device call.  tries: list of (keys, vals).
    devices: a list of GPU ids -> kh_trie_roots_segmented_sharded (contiguous trie ranges
    balanced by slot count, one per device)."""
    keys, vals, seg_off = [], [], [0]
    klen = None
    for ks, vs in tries:
        if len(ks) != len(vs):
            raise MPTException(_lib.KH_EINVAL, "keys/values length mismatch")
        keys += list(ks)
        vals += list(vs)
        seg_off.append(len(keys))
        if ks and klen is None:
            klen = len(ks[0])
    klen = klen or 32
    kb, n = _keys_buf(keys, klen)
    vb, off = _pack(vals)
    so = np.asarray(seg_off, dtype=np.uint64)
    nseg = len(tries)
    out = np.zeros(32 * max(nseg, 1), dtype=np.uint8)
    st = stats if stats is not None else KhStats()
    flags = _lib.KH_HASH_KEYS if hash_keys else 0
    if devices is None:
        check(lib().kh_trie_roots_segmented(kb.ctypes.data, klen, vb.ctypes.data, off.ctypes.data, so.ctypes.data,
                                            nseg, flags, out.ctypes.data, ctypes.byref(st)))
    else:
        dv = np.asarray(list(devices), dtype=np.int32)
        check(lib().kh_trie_roots_segmented_sharded(dv.ctypes.data, len(dv), kb.ctypes.data, klen, vb.ctypes.data,
                                                    off.ctypes.data, so.ctypes.data, nseg, flags, out.ctypes.data,
                                                    ctypes.byref(st)))
    return [out[32 * i:32 * i + 32].tobytes() for i in range(nseg)]


def trie_roots_varkeys(tries, stats=None):
    """Roots of tries over variable-length unhashed keys (0..32 bytes each; a key that
    prefixes others is a branch value).  tries: list of (keys, vals)."""
    keys, vals, seg_off = [], [], [0]
    for ks, vs in tries:
        if len(ks) != len(vs):
            raise MPTException(_lib.KH_EINVAL, "keys/values length mismatch")
        keys += [bytes(k) for k in ks]
        vals += list(vs)
        seg_off.append(len(keys))
    kb, koff = _pack(keys)
    vb, off = _pack(vals)
    so = np.asarray(seg_off, dtype=np.uint64)
    nseg = len(tries)
    out = np.zeros(32 * max(nseg, 1), dtype=np.uint8)
    st = stats if stats is not None else KhStats()
    check(lib().kh_trie_roots_varkeys(kb.ctypes.data, koff.ctypes.data, vb.ctypes.data, off.ctypes.data,
                                      so.ctypes.data, nseg, out.ctypes.data, ctypes.byref(st)))
    return [out[32 * i:32 * i + 32].tobytes() for i in range(nseg)]


def list_roots(lists, stats=None):
    """Roots of list tries: list j's item i is put under rlp(i) (keys made on the device).
    lists: list of lists of serialized items."""
    items, seg_off = [], [0]
    for it in lists:
        items += list(it)
        seg_off.append(len(items))
    ib, off = _pack(items)
    so = np.asarray(seg_off, dtype=np.uint64)
    nseg = len(lists)
    out = np.zeros(32 * max(nseg, 1), dtype=np.uint8)
    st = stats if stats is not None else KhStats()
    check(lib().kh_list_roots(ib.ctypes.data, off.ctypes.data, so.ctypes.data, nseg, out.ctypes.data,
                              ctypes.byref(st)))
    return [out[32 * i:32 * i + 32].tobytes() for i in range(nseg)]


class MptListValidator:
    """validators/MptListValidator.scala:15-46: a block body's list matches its header root."""

    @staticmethod
    def is_valid(hash_, to_validate):
        return list_roots([list(to_validate)])[0] == bytes(hash_)


def trie_root_nodes(keys, vals, hash_keys=False, stats=None):
    """(root, {hash: encoding}) — the root plus every node a fresh node store needs."""
    klen = 32 if not keys else len(keys[0])
    kb, n = _keys_buf(keys, klen)
    vb, off = _pack(list(vals))
    root = np.zeros(32, dtype=np.uint8)
    st = stats if stats is not None else KhStats()
    nn = ctypes.c_uint64(0)
    nl = ctypes.c_uint64(0)
    flags = _lib.KH_HASH_KEYS if hash_keys else 0
    L = lib()
    cap_n, cap_b = 0, 0
    for _ in range(2):
        hs = np.zeros(32 * max(cap_n, 1), dtype=np.uint8)
        rl = np.zeros(max(cap_b, 1), dtype=np.uint8)
        of = np.zeros(cap_n + 1, dtype=np.uint64)
        rc = L.kh_trie_root_nodes(kb.ctypes.data, klen, vb.ctypes.data, off.ctypes.data, n, flags, root.ctypes.data,
                                  hs.ctypes.data, cap_n, rl.ctypes.data, cap_b, of.ctypes.data, ctypes.byref(nn),
                                  ctypes.byref(nl), ctypes.byref(st))
        if rc == _lib.KH_ENOSPC:
            cap_n, cap_b = nn.value, nl.value
            continue
        check(rc)
        nodes = {hs[32 * i:32 * i + 32].tobytes(): rl[of[i]:of[i + 1]].tobytes() for i in range(nn.value)}
        return root.tobytes(), nodes
    raise RuntimeError("kh_trie_root_nodes: size negotiation failed")


class MerklePatriciaTrie:
    """khipu.trie.MerklePatriciaTrie over the device engine (MerklePatriciaTrie.scala:68-558).

    Keys and values are bytes (the reference's ByteArrayEncoder/ByteArraySerializable
    have already been applied, as in GenesisDataLoader.scala:142-146).  With
    ``hash_keys=True`` the key encoder is kec256 (Address.hashedAddressEncoder,
    trie/package.scala hashDataWordSerializable).
    """

    def __init__(self, leaves=None, hash_keys=False, node_storage=None):
        self._leaves = dict(leaves or {})
        self._hash_keys = hash_keys
        self._root = None
        self._changes = None
        self.node_storage = node_storage if node_storage is not None else {}

    def _k(self, key):
        return kec256(key) if self._hash_keys else bytes(key)

    def get(self, key):
        """get (:90-133): the value, or None."""
        return self._leaves.get(self._k(key))

    def put(self, key, value):
        """put (:157-173): returns the trie (the reference returns a new instance)."""
        self._leaves[self._k(key)] = bytes(value)
        self._root = self._changes = None
        return self

    def remove(self, key):
        """remove (:290-315): removing an absent key is a no-op."""
        k = self._k(key)
        if k in self._leaves:
            del self._leaves[k]
            self._root = self._changes = None
        return self

    def update(self, to_remove, to_upsert):
        raise NotImplementedError("Use put/remove")  # :487-489 (UnsupportedOperationException)

    def root_hash(self) -> bytes:
        """rootHash (:78): kec256 of the root encoding; EMPTY_TRIE_HASH when empty."""
        if self._root is None:
            if not self._leaves:
                self._root = EMPTY_TRIE_HASH
            else:
                ks = list(self._leaves.keys())
                vs = [self._leaves[k] for k in ks]
                if all(len(k) == 32 for k in ks):
                    self._root = trie_root(ks, vs)
                else:  # unhashed keys of other lengths (branch values possible)
                    self._root = trie_roots_varkeys([(ks, vs)])[0]
        return self._root

    def changes(self):
        """changes (:549-554) restricted to upserts: {hash: encoding} of every node the
        store needs for the current root (removes are ignored downstream,
        ArchiveNodeStorage.scala:18-20, NodeStorage.scala:16-19)."""
        if self._changes is None:
            if not self._leaves:
                self._root, self._changes = EMPTY_TRIE_HASH, {}
            else:
                ks = list(self._leaves.keys())
                self._root, self._changes = trie_root_nodes(ks, [self._leaves[k] for k in ks])
        return self._changes

    def persist(self):
        """persist (:544-547): write the node set into node_storage."""
        self.node_storage.update(self.changes())
        return self

    def copy(self):
        t = MerklePatriciaTrie(self._leaves, self._hash_keys, self.node_storage)
        t._root, t._changes = self._root, self._changes
        return t

    def __len__(self):
        return len(self._leaves)
