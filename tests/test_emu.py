"""CPU: the device per-thread code (khipu_amd/csrc/trie_ops.h, keccak.h, synth.h),
replayed on the host by tests/emu, against the oracle.  The GPU parity tests run
the same cases through the real kernels."""
import os
import random

import numpy as np
import pytest

from khipu_amd import codec
from tests import cases as C
from tests.emu import emu as E


def _root(r):
    return r[0] if r[1] else codec.EMPTY_TRIE_HASH


@pytest.fixture(params=[0, 1], ids=["leaf3_masked", "leaf3_classified"])
def leaf_mode(request):
    """The early leaf kernel's forms (tests/emu/khst_emu.cc g_leaf_mode)."""
    E.set_leaf_mode(request.param)
    yield request.param
    E.set_leaf_mode(0)


@pytest.fixture(params=[0, 2], ids=["move", "positions"])
def link_mode(request):
    """How the early leaves reach their parents' child records (g_link_mode)."""
    E.set_link_mode(request.param)
    yield request.param
    E.set_link_mode(0)


@pytest.mark.parametrize("case", C.all_cases(), ids=lambda c: c[0])
def test_replay_root_vs_oracle(oracle, case, leaf_mode, link_mode):
    name, keys, vals = case
    res, st = E.build(keys, vals)
    assert _root(res[0]) == oracle.seq_root(keys, vals), name


def test_replay_keccak(oracle):
    r = random.Random(5)
    for L in list(range(0, 280)) + [407, 408, 409, 1000]:
        m = bytes(r.getrandbits(8) for _ in range(L))
        assert E.kec256(m) == oracle.kec256(m)


def test_replay_segmented(oracle):
    tries = C.segmented_case()
    keys = [k for t in tries for k in t[0]]
    vals = [v for t in tries for v in t[1]]
    seg = [i for i, t in enumerate(tries) for _ in t[0]]
    res, _ = E.build(keys, vals, seg=seg, nseg=len(tries))
    for i, (tk, tv) in enumerate(tries):
        exp = oracle.seq_root(tk, tv) if tk else codec.EMPTY_TRIE_HASH
        assert _root(res[i]) == exp, i


@pytest.mark.parametrize("n", [2, 3, 20, 500, 5000])
def test_replay_top_nibble_fold(oracle, n):
    """depth0 = 1 subtries (the multi-GPU shard unit) folded into the root."""
    r = random.Random(n)
    keys = [bytes(r.getrandbits(8) for _ in range(32)) for _ in range(n)]
    vals = [C.storage_value(r) for _ in keys]
    res, _ = E.build(keys, vals, depth0=1)
    ll = np.array([x[1] for x in res], np.uint32)
    if (ll > 0).sum() < 2:
        pytest.skip("root is not a branch")
    hh = np.frombuffer(b"".join(x[0] for x in res), np.uint8).copy()
    ii = np.frombuffer(b"".join(x[2].ljust(32, b"\0") for x in res), np.uint8).copy()
    out = np.zeros(32, np.uint8)
    E.lib().emu_fold16(hh.ctypes.data, ll.ctypes.data, ii.ctypes.data, out.ctypes.data)
    assert out.tobytes() == oracle.seq_root(keys, vals)


def test_replay_genesis(oracle, leaf_mode):
    keys, vals = [], []
    with open(os.path.join(os.path.dirname(__file__), "golden", "genesis_alloc.txt")) as f:
        for line in f:
            a, b = line.split()
            keys.append(oracle.kec256(bytes.fromhex(a)))
            vals.append(codec.account_rlp(0, int(b)))
    res, st = E.build(keys, vals)
    assert _root(res[0]).hex() == "d7f8974fb5ac78d9ac099b9ad5018bedc2ce0a72dad1827a1709da30580f0544"
    assert st[0] == 8893


def test_replay_synth_matches_codec(oracle):
    """csrc/synth.h account bodies == codec.account_rlp of the documented fields."""
    addr, vb, off = E.synth(3, 100, 200)
    for i in range(200):
        body = vb[int(off[i]):int(off[i + 1])].tobytes()
        item = body  # decode the 4 RLP fields with the codec's own framing
        assert body[0] == 0xF8 and body[1] == len(body) - 2
        assert item.endswith(body[-33:])
    # synthetic trie root == oracle
    n = 3000
    addr, vb, off = E.synth(1, 0, n)
    keys = [oracle.kec256(addr[i].tobytes()) for i in range(n)]
    vals = [vb[int(off[i]):int(off[i + 1])].tobytes() for i in range(n)]
    res, _ = E.build(keys, vals)
    assert _root(res[0]) == oracle.seq_root(keys, vals)


def test_nearest_smaller_value_searches():
    """k_ansv's pyramid + SWAR scans == naive nearest-smaller-value definitions."""
    import ctypes
    L = E.lib()
    L.emu_ansv_check.argtypes = [ctypes.c_uint64, ctypes.c_int]
    assert L.emu_ansv_check(7, 150) == 0


def test_tile_topology_matches_whole_array():
    """k_topo_tile (op_tile_ansv / op_tile_chain per tile, the listed boundaries through
    op_ansv / op_chain after it) == op_ansv + op_chain on every boundary: tiles of 1..4096
    boundaries over the boundary values of sorted random keys (uniform, deep, with segment
    breaks).  The emulated builds above run the same tile replay."""
    import ctypes
    L = E.lib()
    L.emu_topo_tile_check.argtypes = [ctypes.c_uint64, ctypes.c_int]
    assert L.emu_topo_tile_check(11, 84) == 0


def test_lane_spread_keccak():
    """keccak_xlane.h (the N1 small-level permutation: 25 lanes per state, two LDS steps per
    round), replayed lane by lane, == keccak.h's one-thread Keccak-f[1600] (which the oracle
    KATs pin) on 300 random states; lanes 25..31 start with garbage and must not leak in."""
    assert E.xlane_check(11, 300) == 0


@pytest.mark.parametrize("kind,depth0", [(1, 0), (1, 1), (2, 0), (2, 1), (3, 1)])
def test_corrupt_boundary_is_an_error_not_a_fault(oracle, kind, depth0):
    """a boundary value outside 0 / depth0 + 1 .. 64 (the r5y fault: a
    speculative build's stale bytes put leaf depths outside 0..63 and the leaf kernel indexed
    past its buffers) is flagged where depths are made -- the early leaves' parent-depth scatter
    (pd_scatter_vals) and the branch records (op_branch_topo) -- and clamped, so no kernel reads
    a depth out of range; the device build returns KH_EINTERNAL at the topology's counter sync.
    Replayed with such a value injected; the same build without it is the oracle's root."""
    r = random.Random(5 + kind)
    keys = [bytes(r.getrandbits(8) for _ in range(32)) for _ in range(300)]
    vals = [C.account_value(r) for _ in keys]
    E.set_leaf_mode(1)
    E.set_link_mode(2)
    try:
        E.set_inject(kind, 17)
        with pytest.raises(AssertionError, match="-9"):
            E.build(keys, vals, depth0=depth0)
    finally:
        E.set_inject(0)
    res, _ = E.build(keys, vals)
    assert res[0][0] == oracle.seq_root(keys, vals)
