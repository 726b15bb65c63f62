"""GPU: the JNI shim (jni/khst_jni.c) end to end through an in-process JNIEnv
(tests/jni_stub/fake_env.c, driven by jni_driver.c): the root from Java arrays (region copies)
and from direct ByteBuffers (no copy) against the oracle, openHost + get (the last put of a
repeated key, an absent key as null) + the idempotent free, and a node missing from the store
thrown as MPTNodeMissingException through the Scala factory Khst.nodeMissing with the missing
hash (the case class has no (String) constructor; Ledger.scala:511/542 match on
its hash and storage)."""
import json
import os
import random
import subprocess

import numpy as np
import pytest

from tests import cases as C

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(tmp_path, keys, vals, klen):
    p = tmp_path / "in.bin"
    voff = np.zeros(len(vals) + 1, np.uint64)
    voff[1:] = np.cumsum([len(v) for v in vals])
    with open(p, "wb") as f:
        f.write(np.uint32(klen).tobytes() + np.uint64(len(keys)).tobytes())
        f.write(b"".join(keys) + voff.tobytes() + b"".join(vals))
    r = subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "tests", "jni_stub")], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    r = subprocess.run([os.path.join(ROOT, "tests", "jni_stub", "jni_driver"), "gpu", str(p)], capture_output=True,
                       text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    return {d["check"]: d for d in map(json.loads, r.stdout.split("\n")[:-1])}


@pytest.mark.parametrize("klen", [32, 20])
def test_jni_roots_get_and_missing_node(tmp_path, oracle, klen):
    rnd = random.Random(41 + klen)
    keys = [bytes(rnd.getrandbits(8) for _ in range(klen)) for _ in range(3000)]
    keys[5] = keys[1]  # a repeated key: the later put wins
    vals = [C.account_value(rnd) for _ in keys]
    got = _run(tmp_path, keys, vals, klen)
    tk = keys if klen == 32 else [oracle.kec256(k) for k in keys]
    want = oracle.seq_root(tk, vals).hex()
    assert got["array_root"]["root"] == want and got["array_root"]["pending"] == 0
    assert got["direct_root"]["root"] == want and got["direct_root"]["pending"] == 0
    assert got["open_host"]["root"] == want and got["open_host"]["handle_ok"] == 1
    assert got["get"]["ok"] == 1, got["get"]
    assert got["free"]["box"] == 0 and got["free"]["pending"] == 0
    m = got["open_nodes_missing"]
    missing = bytes(0x11 * (i + 1) & 0xFF for i in range(32)).hex()
    assert m["handle"] == 0 and m["pending"] == 1, m
    assert m["exc"] == "khipu/trie/MerklePatriciaTrie$MPTNodeMissingException", m
    assert m["factory_calls"] == 1 and m["factory_hash"] == missing and m["missing_out"] == missing, m
