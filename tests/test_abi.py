"""CPU: libkhst.so builds for gfx950, loads, and exports every symbol include/khst.h declares.
No compute calls here (no GPU); the device-free entry points are exercised."""
import ctypes
import os
import re

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared():
    with open(os.path.join(ROOT, "include", "khst.h")) as f:
        src = f.read()
    return sorted(set(re.findall(r"^(?:int|const char\*)\s+(kh_\w+)\s*\(", src, re.M)))


def test_header_symbols_exported():
    import khipu_amd
    from khipu_amd import _lib
    L = khipu_amd.lib()
    declared = _declared()
    assert len(declared) >= 12
    for name in declared:
        assert hasattr(L, name), name
    assert sorted(_lib.EXPORTS) == declared


def test_library_is_gfx950_code_object():
    lib = os.path.join(ROOT, "khipu_amd", "libkhst.so")
    data = open(lib, "rb").read()
    assert b"gfx950" in data


def test_version_and_errors_without_device():
    import khipu_amd
    L = khipu_amd.lib()
    assert L.kh_version().startswith(b"khst")
    assert L.kh_device_count() >= 0


def test_fold_root16_host_path(oracle):
    """kh_fold_root16 is pure host code (same Keccak/RLP code as the device)."""
    import random
    from khipu_amd.device import fold_root16
    from tests.emu import emu as E
    r = random.Random(1)
    keys = [bytes(r.getrandbits(8) for _ in range(32)) for _ in range(300)]
    vals = [bytes([r.randrange(1, 0x80)]) for _ in keys]
    res, _ = E.build(keys, vals, depth0=1)
    hh = np.frombuffer(b"".join(x[0] for x in res), np.uint8).copy()
    ll = np.array([x[1] for x in res], np.uint32)
    ii = np.frombuffer(b"".join(x[2].ljust(32, b"\0") for x in res), np.uint8).copy()
    assert fold_root16(hh, ll, ii) == oracle.seq_root(keys, vals)
    with pytest.raises(khipu_amd_err()):
        fold_root16(hh, np.array([32] + [0] * 15, np.uint32), ii)


def khipu_amd_err():
    from khipu_amd import MPTException
    return MPTException
