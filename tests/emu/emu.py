"""TEST INFRASTRUCTURE ONLY: ctypes wrapper of tests/emu/libkhst_emu.so (host
replay of the device per-thread code, see khst_emu.cc)."""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = os.path.join(_HERE, "libkhst_emu.so")
_lib = None


def lib():
    global _lib
    if _lib is None:
        subprocess.check_call(["make", "-s", "-C", _HERE])
        L = ctypes.CDLL(_LIB)
        vp = ctypes.c_void_p
        L.emu_build.argtypes = [vp, vp, vp, ctypes.c_uint64, vp, ctypes.c_uint64, ctypes.c_uint32, vp, vp, vp, vp]
        L.emu_kec256.argtypes = [vp, ctypes.c_uint64, vp]
        L.emu_synth.argtypes = [ctypes.c_uint32, ctypes.c_uint64, ctypes.c_uint64, vp, vp, vp]
        L.emu_fold16.argtypes = [vp, vp, vp, vp]
        L.emu_node_children.argtypes = [vp, ctypes.c_uint64, ctypes.c_int, vp, vp, vp]
        L.emu_set_leaf_mode.argtypes = [ctypes.c_int]
        L.emu_set_link_mode.argtypes = [ctypes.c_int]
        L.emu_set_inject.argtypes = [ctypes.c_int, ctypes.c_uint64]
        L.emu_xlane_check.argtypes = [ctypes.c_uint64, ctypes.c_int]
        _lib = L
    return _lib


def set_leaf_mode(mode):
    """0 / 1: op_leaf_in3 with the loosest / the lane's own wave bounds."""
    lib().emu_set_leaf_mode(mode)


def set_inject(kind, j=0):
    """a corrupt boundary value (stale bytes, the r5y fault): 1 u[j] = 200 before the leaves'
    parent-depth scatter, 2 the first representative boundary from j set to 70 before the
    branch records, 3 u[j] = 1 before the scatter (invalid under depth0 = 1); 0 off"""
    lib().emu_set_inject(kind, j)


def set_link_mode(mode):
    """0: link slots + copy pass (segmented builds); 2: leaf positions (unsegmented builds)."""
    lib().emu_set_link_mode(mode)


def _buf(b):
    a = np.frombuffer(b, dtype=np.uint8) if len(b) else np.zeros(1, np.uint8)
    return np.ascontiguousarray(a)


def pack(vals):
    off = np.zeros(len(vals) + 1, dtype=np.uint64)
    if vals:
        off[1:] = np.cumsum([len(v) for v in vals])
    return _buf(b"".join(vals) + b"\0" * 16), off


def build(keys32, vals, seg=None, nseg=1, depth0=0):
    """Returns (results, stats): results = list of (hash32, enc_len, inline_bytes)."""
    n = len(keys32)
    kb = _buf(b"".join(keys32) + b"\0" * 16)
    vb, off = pack(vals)
    nres = nseg if seg is not None else (16 if depth0 == 1 else 1)
    oh = np.zeros(32 * nres, np.uint8)
    ol = np.zeros(nres, np.uint32)
    oi = np.zeros(32 * nres, np.uint8)
    st = np.zeros(8, np.uint64)
    sg = np.asarray(seg, dtype=np.uint32) if seg is not None else None
    rc = lib().emu_build(kb.ctypes.data, vb.ctypes.data, off.ctypes.data, n,
                         sg.ctypes.data if sg is not None else None, nseg, depth0,
                         oh.ctypes.data, ol.ctypes.data, oi.ctypes.data, st.ctypes.data)
    assert rc == 0, rc
    res = [(oh[32 * r:32 * r + 32].tobytes(), int(ol[r]), oi[32 * r:32 * r + int(ol[r])].tobytes() if ol[r] < 32 else b"")
           for r in range(nres)]
    return res, st


def kec256(b: bytes) -> bytes:
    out = np.zeros(32, np.uint8)
    buf = _buf(b + b"\0" * 16)
    lib().emu_kec256(buf.ctypes.data, len(b), out.ctypes.data)
    return out.tobytes()


def synth(cfg, first, n):
    addr = np.zeros(20 * n + 16, np.uint8)
    vals = np.zeros(96 * n + 16, np.uint8)
    off = np.zeros(n + 1, np.uint64)
    lib().emu_synth(cfg, first, n, addr.ctypes.data, vals.ctypes.data, off.ctypes.data)
    return addr[:20 * n].reshape(n, 20), vals[:int(off[n])], off


def node_children(value: bytes, kind: int):
    out = np.zeros(512, np.uint8)
    kinds = np.zeros(16, np.uint8)
    n = np.zeros(1, np.uint32)
    buf = _buf(value + b"\0" * 16)
    st = lib().emu_node_children(buf.ctypes.data, len(value), kind, out.ctypes.data, kinds.ctypes.data, n.ctypes.data)
    return st, [(out[32 * i:32 * i + 32].tobytes(), int(kinds[i])) for i in range(int(n[0]))]


def xlane_check(seed, iters):
    """Mismatching state lanes of the lane-spread permutation (keccak_xlane.h, replayed lane
    by lane) against the one-thread permutation (keccak.h) over `iters` random states."""
    return lib().emu_xlane_check(seed, iters)
