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

    def kec256(self, data, off, n):
        t = self.torch
        out = t.empty(32 * max(n, 1), dtype=t.uint8, device=data.device)
        self._sync()
        check(lib().kh_dev_kec256_batch(self.h, _ptr(data), _ptr(off), n, _ptr(out)))
        self._sync()
        return out[:32 * n]

    def build(self, keys, klen, vals, voff, n, seg=None, nseg=1, depth0=0, hash_keys=False):
        """Returns (hash32 [nres,32] uint8, enc_len [nres] uint32, inline [nres,32] uint8, KhStats)."""
        nres = nseg if seg is not None else (16 if depth0 == 1 else 1)
        hh = np.zeros(32 * nres, np.uint8)
        ll = np.zeros(nres, np.uint32)
        ii = np.zeros(32 * nres, np.uint8)
        st = KhStats()
        flags = _lib.KH_HASH_KEYS if hash_keys else 0
        self._sync()
        check(lib().kh_dev_trie_build(self.h, _ptr(keys), klen, _ptr(vals), _ptr(voff), n, _ptr(seg), nseg, depth0,
                                      flags, hh.ctypes.data, ll.ctypes.data, ii.ctypes.data, ctypes.byref(st)))
        return hh.reshape(nres, 32), ll, ii.reshape(nres, 32), st


def fold_root16(hash32x16, len16, inline32x16):
    """Root over 16 capped top-nibble references (kh_fold_root16)."""
    hh = np.ascontiguousarray(hash32x16, dtype=np.uint8).reshape(-1)
    ll = np.ascontiguousarray(len16, dtype=np.uint32)
    ii = np.ascontiguousarray(inline32x16, dtype=np.uint8).reshape(-1)
    out = np.zeros(32, np.uint8)
    check(lib().kh_fold_root16(hh.ctypes.data, ll.ctypes.data, ii.ctypes.data, out.ctypes.data))
    return out.tobytes()
