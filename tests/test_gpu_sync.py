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


def test_verify_nodes_packed_and_duplicate_requests(khst, oracle):
    """kh_verify_nodes_packed (children concatenated in processResponse's order) equals the
    16-slot form and the oracle's batch restatement (or_verify_nodes), with requests listed
    twice under different kinds (requestNodeHashes.toMap: the later one wins) and values
    nobody requested."""
    import ctypes
    import numpy as np
    from khipu_amd._lib import check, lib
    r = random.Random(6)
    values, reqs, kinds = [], [], []
    for name, kind, nodes in C.sync_node_sets(oracle):
        for h, enc in nodes.items():
            values.append(enc)
            reqs.append(h)
            kinds.append(kind)
            if r.random() < 0.1:
                values.append(C.mutate(r, enc))
    for q in range(0, len(reqs), 7):  # duplicates: the later kind wins
        reqs.append(reqs[q])
        kinds.append(2 if kinds[q] == 0 else 0)
    n = len(values)
    data = np.frombuffer(b"".join(values) + bytes(16), np.uint8)
    off = np.concatenate([[0], np.cumsum([len(v) for v in values])]).astype(np.uint64)
    req = np.frombuffer(b"".join(reqs), np.uint8)
    kd = np.array(kinds, np.uint8)
    hh = np.zeros((n, 32), np.uint8)
    match = np.zeros(n, np.int64)
    status = np.zeros(n, np.uint8)
    coff = np.zeros(n + 1, np.uint64)
    child = np.zeros((16 * n, 32), np.uint8)
    ckind = np.zeros(16 * n, np.uint8)
    tot = ctypes.c_uint64()
    check(lib().kh_verify_nodes_packed(data.ctypes.data, off.ctypes.data, n, req.ctypes.data, kd.ctypes.data,
                                       len(reqs), hh.ctypes.data, match.ctypes.data, status.ctypes.data,
                                       coff.ctypes.data, child.ctypes.data, ckind.ctypes.data, 16 * n,
                                       ctypes.byref(tot)))
    ch, cm, cs, cn, cc, ck = oracle.verify_nodes_batch(data, off, req, kd)
    assert (ch == hh).all() and (cm == match).all() and (cs == status).all()
    assert (np.diff(coff) == cn).all() and int(tot.value) == int(cn.sum())
    mask = np.arange(16)[None, :] < cn[:, None]
    t = int(tot.value)
    assert (cc[mask] == child[:t]).all() and (ck[mask] == ckind[:t]).all()
    # a short children buffer: KH_ENOSPC with the total
    rc = lib().kh_verify_nodes_packed(data.ctypes.data, off.ctypes.data, n, req.ctypes.data, kd.ctypes.data,
                                      len(reqs), hh.ctypes.data, match.ctypes.data, status.ctypes.data,
                                      coff.ctypes.data, child.ctypes.data, ckind.ctypes.data, t - 1,
                                      ctypes.byref(tot))
    assert rc == -6 and int(tot.value) == t
    # the 16-slot form on the same batch
    from khipu_amd import sync
    hh2, m2, s2, kids = sync.verify_nodes(values, [sync.NodeHash(h, k) for h, k in zip(reqs, kinds)])
    assert (hh2 == hh).all() and (m2 == match).all() and (s2 == status).all()
    for i in range(n):
        assert [(k.hash, k.kind) for k in kids[i]] == [(cc[i, j].tobytes(), int(ck[i, j])) for j in range(cn[i])]
