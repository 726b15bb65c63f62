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


def _ref_decode(d, pos=0):
    """RLP.decodeWithPos / getItemBounds / slice as the reference runs them
    (rlp/RLP.scala:179-230): `slice` is Arrays.copyOfRange, which ZERO-PADS a range past
    the end, and reading a prefix byte past the end throws (ArrayIndexOutOfBounds ->
    IndexError here)."""
    def sl(a, b):
        return bytes(d[a:b]) + b"\0" * max(0, b - max(a, len(d)))
    p = d[pos]
    if p == 0x80:
        return b"", pos + 1
    if p < 0x80:
        return bytes([p]), pos + 1
    if p <= 0xB7:
        n = p - 0x80
        return sl(pos + 1, pos + 1 + n), pos + 1 + n
    if p < 0xC0:
        ll = p - 0xB7
        n = int.from_bytes(sl(pos + 1, pos + 1 + ll), "big")
        b = pos + 1 + ll
        return sl(b, b + n), b + n
    if p <= 0xF7:
        b, n = pos + 1, p - 0xC0
    else:
        ll = p - 0xF7
        n = int.from_bytes(sl(pos + 1, pos + 1 + ll), "big")
        b = pos + 1 + ll
    items, q = [], b
    while q < b + n:
        it, q = _ref_decode(d, q)
        items.append(it)
    return items, b + n


def test_truncated_items_reference_behaviour(oracle):
    """What the reference does with a TRUNCATED node value, and why kh_verify_nodes may
    reject it instead (status 4, strict decode).  The reference zero-pads a string item that
    runs past the end (copyOfRange) or throws ArrayIndexOutOfBounds when a list item's
    prefix lies past the end; either way the value is not a node encoding.  A NodeData
    value reaches the decoder only after its kec256 matched a REQUESTED hash
    (sync/package.scala:88-95), i.e. it is a preimage of a hash some valid trie node
    produced, and every valid node is well-formed RLP -- so truncated values are
    unreachable in the reference's flow and the two decoders agree on every reachable
    input (test_node_children_real_nodes)."""
    from tests.emu import emu
    leaf = bytes.fromhex("e1a0") + bytes(range(32))  # [HP path (32 B string)]: one item
    trunc_string = leaf[:-5]  # the string runs 5 bytes past the end
    items, _ = _ref_decode(trunc_string)
    assert items == [bytes(range(27)) + b"\0" * 5]  # the reference zero-pads
    trunc_list = bytes([0xC4, 0x82, 0x01])  # the list claims 4 bytes, 2 present
    with pytest.raises(IndexError):  # the reference throws reading the next prefix
        _ref_decode(trunc_list)
    for v in (trunc_string, trunc_list):
        for kind in (0, 2):
            st_o = oracle.node_children(v, kind)[0]
            assert st_o != 0 and emu.node_children(v, kind)[0] == st_o


def test_batch_verify_matches_per_node_decode(oracle):
    """or_verify_nodes (the CPU leg of bench.py --workload verify) equals the per-node
    restatement: kec256 of each value, the last request of a hash wins
    (requestNodeHashes.toMap, sync/package.scala:85), children of matched trie nodes only."""
    import numpy as np
    r = random.Random(4)
    values, reqs, kinds = [], [], []
    for name, kind, nodes in _sets(oracle):
        for h, enc in nodes.items():
            values.append(enc)
            reqs.append(h)
            kinds.append(kind)
            if r.random() < 0.1:
                values.append(C.mutate(r, enc))  # not requested
    reqs.append(reqs[0])  # a duplicate request: the later kind (EvmcodeHash) wins
    kinds.append(3)
    data = np.frombuffer(b"".join(values) + bytes(16), np.uint8)
    off = np.concatenate([[0], np.cumsum([len(v) for v in values])]).astype(np.uint64)
    req = np.frombuffer(b"".join(reqs), np.uint8)
    hh, match, status, nchild, child, ckind = oracle.verify_nodes_batch(data, off, req, np.array(kinds, np.uint8))
    last = {h: i for i, h in enumerate(reqs)}
    for i, v in enumerate(values):
        h = oracle.kec256(v)
        assert hh[i].tobytes() == h
        assert match[i] == last.get(h, -1)
        if match[i] < 0 or kinds[match[i]] == 3:
            assert nchild[i] == 0 and status[i] == 0
            continue
        st, ch = oracle.node_children(v, kinds[match[i]])
        assert status[i] == st
        assert [(child[i, j].tobytes(), int(ckind[i, j])) for j in range(nchild[i])] == ch
