"""Fast-sync NodeData verification: the decode shared by the HIP
kernel (khipu_amd/csrc/nodedata.h, here through the host replay) against the oracle's
restatement of PV63's MptNode decoder + NodeDatasRequest's child lists
(PV63.scala:96-127, sync/package.scala:127-165), on real trie nodes and on random
corruptions of them."""
import random

import pytest

from tests import cases as C


def _sets(oracle):
    return C.sync_node_sets(oracle)


def test_node_children_real_nodes(oracle):
    from tests.emu import emu
    n_kids = 0
    for name, kind, nodes in _sets(oracle):
        assert len(nodes) > 20, name
        for h, enc in nodes.items():
            want = oracle.node_children(enc, kind)
            assert want[0] == 0, (name, enc.hex())
            got = emu.node_children(enc, kind)
            assert got == want, (name, enc.hex())
            n_kids += len(want[1])
            # the other interpretation (storage vs state) too
            other = 2 if kind == 0 else 0
            assert emu.node_children(enc, other) == oracle.node_children(enc, other)
    assert n_kids > 300


def test_state_leaf_children_kinds(oracle):
    """A contract account leaf lists its code hash (EvmcodeHash) then its storage
    root (StorageRootHash); an ordinary account lists none."""
    from khipu_amd import codec
    from tests.emu import emu
    sr, ch = bytes(range(32)), bytes(range(32, 64))
    t = oracle.Trie()
    t.put(b"\x11" * 32, codec.account_rlp(1, 2, state_root=sr, code_hash=ch))
    t.put(b"\x22" * 32, codec.account_rlp(1, 2))
    nodes = t.reachable()
    leaves = [e for e in nodes.values() if any(k == 3 for _, k in oracle.node_children(e, 0)[1])]
    assert len(leaves) == 1
    st, kids = emu.node_children(leaves[0], 0)
    assert st == 0 and kids == [(ch, 3), (sr, 1)]
    # the root branch lists its two (hashed) children as state-trie nodes
    root = nodes[t.root_hash()]
    st, kids = emu.node_children(root, 0)
    assert st == 0 and len(kids) == 2 and all(k == 0 for _, k in kids)


def test_node_children_fuzz(oracle):
    from tests.emu import emu
    r = random.Random(5)
    seen = set()
    for name, kind, nodes in _sets(oracle):
        encs = list(nodes.values())
        for _ in range(1500):
            bad = C.mutate(r, r.choice(encs))
            want = oracle.node_children(bad, kind)
            got = emu.node_children(bad, kind)
            assert got == want, (name, bad.hex())
            seen.add(want[0])
    for _ in range(300):  # random bytes
        b = bytes(r.getrandbits(8) for _ in range(r.randrange(0, 80)))
        assert emu.node_children(b, 0) == oracle.node_children(b, 0), b.hex()
    assert {0, 1, 2, 4} <= seen, seen


@pytest.mark.parametrize("kind", [0, 2])
def test_evmcode_and_unknown_are_not_decoded(oracle, kind):
    from tests.emu import emu
    assert emu.node_children(b"\x60\x00", 3) == (0, [])
    assert oracle.node_children(b"\x60\x00", 3) == (0, [])
    assert emu.node_children(b"\xc0", kind) == oracle.node_children(b"\xc0", kind)
