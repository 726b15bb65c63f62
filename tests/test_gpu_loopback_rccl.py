"""GPU: the RCCL branch of kh_trie_root_sharded (csrc/sharded.h: ncclCommInitAll, the grouped
ncclSend / ncclRecv of keys on the shards' build streams, then lengths and values on their
exchange streams, the received value offsets scanned behind them) executed on the one-GPU box
through the in-process loopback RCCL (tests/loopback), with the device list
[0] * N and KH_SHARD_RCCL.  Every root is checked against the oracle (small cases) or the pinned
configs[4] root (100M), against the device-copy exchange of the same call and against the
single-GPU build; the loopback's counters show that every block went through ncclSend/ncclRecv.

This is the path the JVM takes for the 8-GPU root, whose fold follows
MerklePatriciaTrie.scala:169.  Edge cases: every key under one top nibble (one owner holds
everything, the others receive nothing), owners without keys, N = 2 / 3 / 8 / 16, raw and
hashed keys."""
import json
import os
import random
import subprocess
import sys

import numpy as np
import pytest

from tests import cases as C

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _lib():
    r = subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "tests", "loopback")], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr


def _cases():
    rnd = random.Random(77)
    out = []

    def add(keys, vals, klen, hk, world, name):
        out.append((name, keys, vals, klen, hk, world))

    addrs = [bytes(rnd.getrandbits(8) for _ in range(20)) for _ in range(4000)]
    add(addrs, [C.account_value(rnd) for _ in addrs], 20, 1, 8, "hashed_w8")
    add(addrs, [C.account_value(rnd) for _ in addrs], 20, 1, 3, "hashed_w3")
    raw = [bytes(rnd.getrandbits(8) for _ in range(32)) for _ in range(3000)]
    add(raw, [C.account_value(rnd) for _ in raw], 32, 0, 16, "raw_w16")
    one = [bytes([0x30 | rnd.getrandbits(4)]) + bytes(rnd.getrandbits(8) for _ in range(31)) for _ in range(2000)]
    add(one, [C.account_value(rnd) for _ in one], 32, 0, 8, "single_nibble_w8")
    two = [bytes([rnd.choice((0x05, 0xF7))]) + bytes(rnd.getrandbits(8) for _ in range(31)) for _ in range(2000)]
    add(two, [C.account_value(rnd) for _ in two], 32, 0, 8, "two_owners_of_8")
    dup = raw[:500] + raw[:100]  # repeated keys: the later put wins across the exchange
    add(dup, [C.account_value(rnd) for _ in dup], 32, 0, 2, "repeats_w2")
    add(raw[:1], [b"\x01"], 32, 0, 4, "one_key_w4")
    return out


def _write(tmp_path, cases):
    arrs = {}
    for i, (_, keys, vals, klen, hk, world) in enumerate(cases):
        voff = np.zeros(len(vals) + 1, np.uint64)
        voff[1:] = np.cumsum([len(v) for v in vals])
        arrs[f"keys_{i}"] = np.frombuffer(b"".join(keys), np.uint8).reshape(len(keys), klen)
        arrs[f"vals_{i}"] = np.frombuffer(b"".join(vals) + b"\0", np.uint8)
        arrs[f"voff_{i}"] = voff
        arrs[f"meta_{i}"] = np.array([klen, hk, world], np.int64)
    p = tmp_path / "cases.npz"
    np.savez(p, **arrs)
    return p


def _run(path, full=False, timeout=180):
    cmd = [sys.executable, os.path.join(ROOT, "tests", "loopback", "run_sharded.py"), str(path)] + (["--full"] if full else [])
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    return [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]


def test_rccl_branch_through_loopback(tmp_path, oracle):
    _lib()
    cases = _cases()
    got = _run(_write(tmp_path, cases))
    assert len(got) == len(cases)
    for (name, keys, vals, klen, hk, world), g in zip(cases, got):
        tk = [oracle.kec256(k) for k in keys] if hk else keys
        want = oracle.seq_root(tk, vals).hex()
        assert g["loopback"] == want, name
        assert g["copies"] == want and g["single"] == want, name
        # the RCCL branch really ran: every non-empty (source, owner) block went through a
        # matched send/recv (at least the keys' group), and the device-copy call used none
        assert g["ops"] > 0 and g["bytes"] > 0, (name, g)
        assert g["ops_copy_path"] == 0, (name, g)


@pytest.mark.timeout(900)
def test_rccl_branch_config4_100m(tmp_path):
    """configs[4] at size over the loopback: 100M synthetic accounts in eight 12.5M slices,
    every (source, owner) block exchanged by ncclSend/ncclRecv, root == the pinned root."""
    _lib()
    np.savez(tmp_path / "none.npz", none=np.zeros(1))
    got = _run(tmp_path / "none.npz", full=True, timeout=800)
    g = got[-1]
    assert g["case"] == "config4_100m"
    assert g["loopback"] == g["pinned"], g
    # 8 sources x 8 owners: keys (group 1), lengths and values (group 2); 100M x 32 B of keys at least
    assert g["groups"] == 2 and g["bytes"] >= 100_000_000 * (32 + 8), g
