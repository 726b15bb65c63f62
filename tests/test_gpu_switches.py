"""GPU parity of every measurement switch the library reads (KHST_* environment variables,
read per call; the defaults are the measured winners).  Each alternative
schedule or kernel stays a correct engine: under each switch the edge cases give the
khipu-faithful oracle's roots, a segmented build its storage roots, raw keys with runs of
equal 32-bit sort prefixes (ties) and repeats the CPU batch builder's root, and a 200k-account
device build the batch builder's root and permutation count."""
import random

import numpy as np
import pytest

from tests import cases as C

pytestmark = pytest.mark.gpu

SWITCHES = [
    "KHST_TIE_ONE=1",
    "KHST_SPEC=0",
    "KHST_PUBLISH_ONE=1",
    "KHST_LEAF_LINKS=1",
    "KHST_LEAF_LINKS=1,KHST_TOPO_TILE=0",
    "KHST_BRANCH=rescan",
    "KHST_BRANCH=coop",
    "KHST_LEAF_POS=0",
    "KHST_LEAF_POS=0,KHST_MOVE_SPLIT=1",
    "KHST_LEAF=v2",
    "KHST_LEAF=sorted",
    "KHST_SEG_CK=0",
    "KHST_TOPO_BPC=0",
    "KHST_TOPO_BPC=2",
    "KHST_TOPO_TILE=0",
    "KHST_TOPO_TILE=1",
    "KHST_TOPO_TILE=2",
    "KHST_TOPO_TILE=3",
    "KHST_PD=sep",
    "KHST_PD=first",
    "KHST_PD=sep,KHST_TOPO_TILE=0",
    "KHST_BRANCH_BS=64",
    "KHST_BRANCH_SMALL=0",
    "KHST_XL_LEVEL=0",
    "KHST_XL_LEVEL=1000000,KHST_SMALL_LEVEL=1000000",
    "KHST_SMALL_LEVEL=0",
    "KHST_LEAF_PRIO=hi",
]


def _tie_keys(seed, n):
    r = random.Random(seed)
    keys = []
    while len(keys) < n:
        pre = bytes(r.getrandbits(8) for _ in range(4))
        keys += [pre + bytes(r.getrandbits(8) for _ in range(28)) for _ in range(r.randint(2, 70))]
    keys += [keys[r.randrange(len(keys))] for _ in range(n // 50)]  # repeats: the last put wins
    r.shuffle(keys)
    return keys, [bytes([r.getrandbits(8) | 1]) * r.choice([1, 5, 40, 80]) for _ in keys]


@pytest.mark.parametrize("switch", SWITCHES)
def test_switch_vs_oracle(khst, oracle, switch, monkeypatch):
    for kv in switch.split(","):
        k, v = kv.split("=")
        monkeypatch.setenv(k, v)
    for name, keys, vals in C.all_cases(big=False):
        assert khst.trie_root(keys, vals) == oracle.seq_root(keys, vals), (switch, name)
    tries = C.segmented_case()
    for (ks, vs), g in zip(tries, khst.trie_roots(tries)):
        assert g == (oracle.seq_root(ks, vs) if ks else khst.EMPTY_TRIE_HASH), switch
    keys, vals = _tie_keys(3, 30_000)
    assert khst.trie_root(keys, vals) == oracle.batch_root(keys, vals, nthreads=4), switch
    from khipu_amd.device import Ctx
    ctx = Ctx(0)  # a fresh context: KHST_LEAF_PRIO is read when its streams are made
    n = 200_000
    addr, dv, voff = ctx.synth_accounts(1, 0, n)
    hh, _, _, st = ctx.build(addr, 20, dv, voff, n, hash_keys=True)
    a = addr[:20 * n].cpu().numpy()
    vo = voff.cpu().numpy().astype(np.uint64)
    roots, bst = oracle.batch_roots(a, (dv[:int(vo[-1])].cpu().numpy(), vo), klen=20, hash_keys=True)
    assert hh[0].tobytes() == roots[0] and st.n_node_perms == bst["node_perms"], switch
