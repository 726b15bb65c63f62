"""CPU: the hot kernels' code placement in the built library (scripts/code_align.py).

The VALU-bound kernels run 10-15 % faster when nearly all of their 8-byte VALU instructions sit
at addresses 4 mod 8 than when the same code sits 4 bytes off (key hashing 10.3 vs 11.8 ms, the
leaf kernel 13.4 vs 14.7 ms at 100M: profiles/r8d_layout_bisect_ab_100m.json,
r8k_leaf_shift_ab_100m.json).  The library is built so that they do (two compilation units,
loop heads aligned to 64 bytes in one: __graft_entry__.UNITS); an edit that shifts a kernel's
code by 4 bytes flips the fraction below 0.2 and fails here instead of in a bench line."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "khipu_amd", "libkhst.so")
sys.path.insert(0, os.path.join(ROOT, "scripts"))

HOT = {  # kernel (mangled-name part) -> the least fraction at 4 mod 8 it is built with
    "_Z9k_leaf_in": 0.85,
    "_Z14k_hash_keys_ckILb1E": 0.85,
    "_Z14k_branch_fusedILi4E": 0.7,
    "_Z14k_branch_fusedILi6E": 0.7,
}


def test_hot_kernels_keep_their_placement():
    if not os.path.exists(LIB):
        pytest.skip("libkhst.so not built")
    import code_align as C
    try:
        ks = C.kernels(C.disassemble(LIB))
    except (OSError, Exception) as e:  # (objcopy / the ROCm LLVM tools absent)
        pytest.skip(f"disassembly unavailable: {e}")
    for part, floor in HOT.items():
        syms = [s for s in ks if s.startswith(part)]
        assert syms, part
        v8, v8m = C.stats(ks[syms[0]])
        assert v8 > 1000 and v8m / v8 >= floor, (syms[0], v8, round(v8m / v8, 3))
