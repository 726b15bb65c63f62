"""ORACLE — TEST INFRASTRUCTURE ONLY.

ctypes wrapper over oracle/liboracle.so, the CPU restatement of khipu's
Keccak-256 / RLP / hex-prefix / MerklePatriciaTrie (see khipu_oracle.cc for the
reference file:line each function follows).  Only tests/, __graft_entry__.smoke()
and bench.py's cpu_baseline leg may import this module, and only as the checker.
The product path (khipu_amd/, libkhst.so) never imports or calls it.
"""
import ctypes
import os
import subprocess

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "liboracle.so")
_lib = None


def build():
    subprocess.check_call(["make", "-s", "-C", _HERE])


def lib():
    global _lib
    if _lib is None:
        srcs = [os.path.join(_HERE, f) for f in ("khipu_oracle.cc", "batch_root.cc")]
        if not os.path.exists(_LIB_PATH) or any(os.path.exists(s) and os.path.getmtime(_LIB_PATH) < os.path.getmtime(s)
                                                for s in srcs):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        u8p = ctypes.c_char_p
        L.or_kec256.argtypes = [u8p, ctypes.c_uint64, ctypes.c_void_p]
        L.or_keccak256_pad.argtypes = [u8p, ctypes.c_uint64, ctypes.c_uint8, ctypes.c_void_p]
        L.or_last_error.restype = ctypes.c_char_p
        L.or_perm_count.restype = ctypes.c_uint64
        for f in ("or_rlp_str", "or_rlp_list"):
            getattr(L, f).argtypes = [u8p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_uint64]
            getattr(L, f).restype = ctypes.c_int64
        L.or_hp_encode.argtypes = [u8p, ctypes.c_uint64, ctypes.c_int, ctypes.c_void_p, ctypes.c_uint64]
        L.or_hp_encode.restype = ctypes.c_int64
        L.or_trie_new.restype = ctypes.c_void_p
        L.or_trie_free.argtypes = [ctypes.c_void_p]
        L.or_trie_put.argtypes = [ctypes.c_void_p, u8p, ctypes.c_uint64, u8p, ctypes.c_uint64]
        L.or_trie_remove.argtypes = [ctypes.c_void_p, u8p, ctypes.c_uint64]
        L.or_trie_get.argtypes = [ctypes.c_void_p, u8p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_uint64]
        L.or_trie_get.restype = ctypes.c_int64
        L.or_trie_root.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
        L.or_trie_persist.argtypes = [ctypes.c_void_p]
        L.or_trie_reopen.argtypes = [ctypes.c_void_p]
        L.or_trie_updated_count.argtypes = [ctypes.c_void_p]
        L.or_trie_updated_count.restype = ctypes.c_uint64
        L.or_trie_updated_dump.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64,
                                           ctypes.c_void_p]
        L.or_trie_reachable.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p,
                                        ctypes.c_uint64, ctypes.c_void_p]
        L.or_trie_reachable.restype = ctypes.c_int64
        L.or_node_children.argtypes = [u8p, ctypes.c_uint64, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                                        ctypes.c_void_p]
        L.or_node_children.restype = ctypes.c_int
        L.or_seq_root.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p,
                                  ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int, ctypes.c_void_p]
        vp, u64 = ctypes.c_void_p, ctypes.c_uint64
        L.or_batch_roots.argtypes = [vp, vp, u64, vp, vp, u64, vp, u64, ctypes.c_int, ctypes.c_int, vp, vp]
        L.or_batch_last_error.restype = ctypes.c_char_p
        L.or_batch_kec256.argtypes = [u8p, u64, vp]
        L.or_verify_nodes.argtypes = [vp, vp, u64, vp, vp, u64, vp, vp, vp, vp, vp, vp]
        _lib = L
    return _lib


def kec256(data: bytes) -> bytes:
    out = ctypes.create_string_buffer(32)
    lib().or_kec256(data, len(data), out)
    return out.raw


def keccak256_pad(data: bytes, pad: int) -> bytes:
    out = ctypes.create_string_buffer(32)
    lib().or_keccak256_pad(data, len(data), pad, out)
    return out.raw


def _call_buf(fn, data, *extra):
    cap = 64 + 2 * len(data)
    out = ctypes.create_string_buffer(cap)
    n = fn(data, len(data), *extra, out, cap)
    assert n >= 0
    return out.raw[:n]


def rlp_str(b: bytes) -> bytes:
    return _call_buf(lib().or_rlp_str, b)


def rlp_list(payload: bytes) -> bytes:
    return _call_buf(lib().or_rlp_list, payload)


def hp_encode(nibbles: bytes, is_leaf: bool) -> bytes:
    return _call_buf(lib().or_hp_encode, nibbles, 1 if is_leaf else 0)


class OracleError(RuntimeError):
    pass


class Trie:
    """khipu-faithful sequential MerklePatriciaTrie (MerklePatriciaTrie.scala:68-558)."""

    def __init__(self):
        self._t = lib().or_trie_new()

    def __del__(self):
        if getattr(self, "_t", None):
            lib().or_trie_free(self._t)
            self._t = None

    def _chk(self, rc):
        if rc != 0:
            raise OracleError(lib().or_last_error().decode())

    def put(self, k: bytes, v: bytes):
        self._chk(lib().or_trie_put(self._t, k, len(k), v, len(v)))
        return self

    def remove(self, k: bytes):
        self._chk(lib().or_trie_remove(self._t, k, len(k)))
        return self

    def get(self, k: bytes):
        buf = ctypes.create_string_buffer(4096)
        n = lib().or_trie_get(self._t, k, len(k), buf, 4096)
        if n == -2:
            return None
        if n < 0:
            raise OracleError(lib().or_last_error().decode())
        return buf.raw[:n]

    def root_hash(self) -> bytes:
        out = ctypes.create_string_buffer(32)
        lib().or_trie_root(self._t, out)
        return out.raw

    def persist(self):
        lib().or_trie_persist(self._t)
        return self

    def reopen(self):
        lib().or_trie_reopen(self._t)
        return self

    def updated(self):
        """dict hash -> encoding of the Updated log entries (the write-back set)."""
        n = lib().or_trie_updated_count(self._t)
        hs = ctypes.create_string_buffer(32 * max(n, 1))
        cap = 1024 * max(n, 1)
        enc = ctypes.create_string_buffer(cap)
        off = (ctypes.c_uint64 * (n + 1))()
        assert lib().or_trie_updated_dump(self._t, hs, enc, cap, off) == 0
        return {hs.raw[32 * i:32 * i + 32]: enc.raw[off[i]:off[i + 1]] for i in range(n)}

    def reachable(self):
        """dict hash -> encoding for every node reachable from the root with encoding >= 32 B, plus the root."""
        n = lib().or_trie_reachable(self._t, None, 0, None, 0, None)
        if n < 0:
            raise OracleError(lib().or_last_error().decode())
        hs = ctypes.create_string_buffer(32 * max(n, 1))
        cap = 600 * max(n, 1)
        enc = ctypes.create_string_buffer(cap)
        off = (ctypes.c_uint64 * (n + 1))()
        m = lib().or_trie_reachable(self._t, hs, n, enc, cap, off)
        assert m == n
        return {hs.raw[32 * i:32 * i + 32]: enc.raw[off[i]:off[i + 1]] for i in range(n)}


def seq_root(keys, vals, dels=None, mode=0) -> bytes:
    """Sequential root over a batch of puts (and removes where dels[i]) in order.

    mode 0: TrieAccounts.flush pattern (TrieAccounts.scala:22-28), one instance.
    mode 1: GenesisDataLoader pattern (GenesisDataLoader.scala:139-147).
    mode | 2: every key is kec256 of the given bytes, hashed in C inside the loop.
    keys: list of equal-length bytes; vals: list of bytes.
    """
    import numpy as np
    n = len(keys)
    klen = len(keys[0]) if n else 32
    kb = b"".join(keys)
    vb = b"".join(vals)
    off = np.zeros(n + 1, dtype=np.uint64)
    if n:
        off[1:] = np.cumsum([len(v) for v in vals])
    d = None
    if dels is not None:
        d = np.asarray(dels, dtype=np.uint8)
    out = ctypes.create_string_buffer(32)
    rc = lib().or_seq_root(kb, klen, vb if vb else None, off.ctypes.data,
                           d.ctypes.data if d is not None else None, n, mode, out)
    if rc != 0:
        raise OracleError(lib().or_last_error().decode())
    return out.raw


def seq_root_packed(keys_u8, klen, vals_u8, voff_u64, n, mode=0) -> bytes:
    """Same as seq_root over numpy buffers (keys n*klen bytes, vals packed with voff[n+1])."""
    out = ctypes.create_string_buffer(32)
    rc = lib().or_seq_root(keys_u8.ctypes.data, klen, vals_u8.ctypes.data, voff_u64.ctypes.data, None, n, mode, out)
    if rc != 0:
        raise OracleError(lib().or_last_error().decode())
    return out.raw


BATCH_STATS = ("leaves", "branches", "extensions", "node_hashes", "node_perms", "key_perms", "inline", "distinct")


def _np_u8(x):
    import numpy as np
    if isinstance(x, (bytes, bytearray)):
        return np.frombuffer(bytes(x) + b"\0" * 8, np.uint8)
    return np.ascontiguousarray(x, dtype=np.uint8).reshape(-1)


def batch_roots(keys, vals, klen=None, seg_off=None, hash_keys=False, nthreads=None):
    """Independent multi-threaded batch builder (oracle/batch_root.cc): roots of the
    tries holding put(keys[i], vals[i]) in order (later puts win).

    keys: list of bytes (any lengths: list tries), or a uint8 array of n*klen;
    vals: list of bytes, or (uint8 array, uint64 offsets[n+1]);
    seg_off: None (one trie) or offsets[nseg+1] from 0 to n (many independent tries).
    Returns (list of 32-byte roots, stats dict)."""
    import numpy as np
    nthreads = nthreads or min(16, os.cpu_count() or 1)
    koff = None
    if isinstance(keys, np.ndarray):
        kb = _np_u8(keys)
        n = kb.size // klen
    else:
        keys = list(keys)
        n = len(keys)
        kb = _np_u8(b"".join(keys))
        lens = {len(k) for k in keys}
        if len(lens) > 1 or klen is None:
            koff = np.zeros(n + 1, np.uint64)
            koff[1:] = np.cumsum([len(k) for k in keys])
            klen = 0
    if isinstance(vals, tuple):
        vb, voff = _np_u8(vals[0]), np.ascontiguousarray(vals[1], dtype=np.uint64)
    else:
        vals = list(vals)
        vb = _np_u8(b"".join(vals))
        voff = np.zeros(len(vals) + 1, np.uint64)
        voff[1:] = np.cumsum([len(v) for v in vals])
    so = None if seg_off is None else np.ascontiguousarray(seg_off, dtype=np.uint64)
    nseg = 1 if so is None else len(so) - 1
    roots = np.zeros(32 * max(nseg, 1), np.uint8)
    st = np.zeros(8, np.uint64)
    rc = lib().or_batch_roots(kb.ctypes.data, None if koff is None else koff.ctypes.data, klen or 0, vb.ctypes.data,
                              voff.ctypes.data, n, None if so is None else so.ctypes.data, nseg,
                              1 if hash_keys else 0, nthreads, roots.ctypes.data, st.ctypes.data)
    if rc != 0:
        raise OracleError(lib().or_batch_last_error().decode())
    return [roots[32 * i:32 * i + 32].tobytes() for i in range(nseg)], dict(zip(BATCH_STATS, map(int, st)))


def batch_root(keys, vals, **kw) -> bytes:
    return batch_roots(keys, vals, **kw)[0][0]


def batch_kec256(data: bytes) -> bytes:
    out = ctypes.create_string_buffer(32)
    lib().or_batch_kec256(data, len(data), out)
    return out.raw


def perm_count() -> int:
    return lib().or_perm_count()


def perm_reset():
    lib().or_perm_reset()


def node_children(value: bytes, kind: int):
    """PV63 decode + NodeDatasRequest child lists of one NodeData value
    (blockchain/sync/package.scala:127-165): (status, [(hash32, kind), ...])."""
    out = ctypes.create_string_buffer(512)
    kinds = ctypes.create_string_buffer(16)
    n = ctypes.c_uint32()
    st = lib().or_node_children(value, len(value), kind, out, kinds, ctypes.byref(n))
    return st, [(out.raw[32 * i:32 * i + 32], kinds.raw[i]) for i in range(n.value)]


def verify_nodes_batch(data, off, req32, req_kind):
    """NodeDatasRequest.processResponse over one batch on one core (or_verify_nodes): numpy
    inputs as kh_verify_nodes takes them; returns (hash32 [n,32], match [n], status [n],
    nchild [n], child32 [n,16,32], child_kind [n,16])."""
    import numpy as np
    n = len(off) - 1
    nreq = len(req_kind)
    data = np.ascontiguousarray(data, np.uint8)
    off = np.ascontiguousarray(off, np.uint64)
    req32 = np.ascontiguousarray(req32, np.uint8)
    req_kind = np.ascontiguousarray(req_kind, np.uint8)
    hh = np.zeros((max(n, 1), 32), np.uint8)
    match = np.zeros(max(n, 1), np.int64)
    status = np.zeros(max(n, 1), np.uint8)
    nchild = np.zeros(max(n, 1), np.uint8)
    child = np.zeros((max(n, 1), 16, 32), np.uint8)
    ckind = np.zeros((max(n, 1), 16), np.uint8)
    rc = lib().or_verify_nodes(data.ctypes.data, off.ctypes.data, n, req32.ctypes.data, req_kind.ctypes.data, nreq,
                               hh.ctypes.data, match.ctypes.data, status.ctypes.data, nchild.ctypes.data,
                               child.ctypes.data, ckind.ctypes.data)
    assert rc == 0
    return hh[:n], match[:n], status[:n], nchild[:n], child[:n], ckind[:n]
