"""GPU parity of fast-sync NodeData verification (kh_verify_nodes)
against the oracle's restatement of PV63 decoding + NodeDatasRequest child lists."""
import random

import pytest

from tests import cases as C

pytestmark = pytest.mark.gpu


def test_verify_nodes_vs_oracle(khst, oracle):
    from khipu_amd import sync
    r = random.Random(2)
    values, reqs, want = [], [], []
    for name, kind, nodes in C.sync_node_sets(oracle):
        for h, enc in nodes.items():
            values.append(enc)
            reqs.append(sync.NodeHash(h, kind))
            want.append(oracle.node_children(enc, kind))
            if r.random() < 0.2:  # corrupted copies: hash no longer matches -> not decoded
                values.append(C.mutate(r, enc))
                want.append(None)
    code = bytes(r.getrandbits(8) for _ in range(5000))  # an EVM code value (long message)
    values.append(code)
    reqs.append(sync.NodeHash(oracle.kec256(code), sync.EVMCODE))
    want.append((0, []))
    hh, match, status, kids = sync.verify_nodes(values, reqs)
    for i, v in enumerate(values):
        assert hh[i].tobytes() == oracle.kec256(v)
        if want[i] is None:
            assert match[i] == -1 or reqs[match[i]].hash == oracle.kec256(v)
            continue
        assert reqs[match[i]].hash == hh[i].tobytes()
        assert int(status[i]) == want[i][0]
        assert [(k.hash, k.kind) for k in kids[i]] == want[i][1]


def test_verify_nodes_malformed_matched(khst, oracle):
    """Corrupted node bytes requested under their own hash: the status must equal
    the oracle's (reference exception -> status code)."""
    from khipu_amd import sync
    r = random.Random(9)
    values, reqs = [], []
    for name, kind, nodes in C.sync_node_sets(oracle):
        encs = list(nodes.values())
        for _ in range(400):
            bad = C.mutate(r, r.choice(encs))
            values.append(bad)
            reqs.append(sync.NodeHash(oracle.kec256(bad), kind))
    hh, match, status, kids = sync.verify_nodes(values, reqs)
    for i, v in enumerate(values):
        st, ch = oracle.node_children(v, reqs[i].kind)
        assert match[i] >= 0 and int(status[i]) == st, v.hex()
        assert [(k.hash, k.kind) for k in kids[i]] == ch


def test_process_response(khst, oracle):
    """NodeDatasRequest.processResponse bookkeeping (sync/package.scala:81-125)."""
    from khipu_amd import sync
    sets = C.sync_node_sets(oracle)
    state = list(sets[0][2].items())[:10]
    stor = list(sets[1][2].items())[:5]
    reqs = [sync.NodeHash(h, sync.STATE_NODE) for h, _ in state] + \
           [sync.NodeHash(h, sync.CONTRACT_NODE) for h, _ in stor] + [sync.NodeHash(b"\x01" * 32, sync.EVMCODE)]
    req = sync.NodeDatasRequest("peer", reqs)
    assert req.process_response([]) is None
    vals = [e for _, e in state[:7]] + [e for _, e in stor] + [b"unrequested"]
    resp = req.process_response(vals)
    assert resp.n_downloaded_nodes == 12
    assert resp.remaining_hashes == reqs[7:10] + reqs[15:]
    want_kids = []
    for _, e in state[:7]:
        want_kids += oracle.node_children(e, 0)[1]
    for _, e in stor:
        want_kids += oracle.node_children(e, 2)[1]
    assert [(k.hash, k.kind) for k in resp.children_hashes] == want_kids
    assert [h for h, _ in resp.received_accounts] == [h for h, _ in state[:7]][::-1]  # prepended (::)
    assert [h for h, _ in resp.received_storages] == [h for h, _ in stor][::-1]
    bad = bytes.fromhex("c3010203")  # a 3-item list requested as a state node
    with pytest.raises(sync.NodeDataError):
        sync.NodeDatasRequest("p", [sync.NodeHash(oracle.kec256(bad), sync.STATE_NODE)]).process_response([bad])
