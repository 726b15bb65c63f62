"""kh_trie_root_sharded (SURVEY §8e through the C ABI): the multi-GPU root for a caller in
one process (the JVM), against the single-GPU build and the oracle.

The test box has one GPU: devices [0] runs the RCCL transport (a one-device
communicator: every block is a self send/recv), and device lists that repeat 0 run 2-16
shards on it (the same partition / exchange layout / per-owner builds / fold, with device
copies as the transport) -- the shard logic at every N the driver's 8-GPU node uses."""
import random

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

EMPTY = bytes.fromhex("56e81f171bcc55a6ff8345e692c0f86e5b48e01b996cadc001622fb5e363b421")
GENESIS_ROOT = "d7f8974fb5ac78d9ac099b9ad5018bedc2ce0a72dad1827a1709da30580f0544"


def _rand(n, seed, top=None):
    r = np.random.default_rng(seed)
    keys = r.integers(0, 256, (n, 32), dtype=np.uint8)
    if top is not None:
        keys[:, 0] = (keys[:, 0] & 0x0F) | (top << 4)
    lens = r.integers(1, 120, n)
    voff = np.zeros(n + 1, np.uint64)
    voff[1:] = np.cumsum(lens)
    vals = r.integers(0, 256, int(voff[-1]) + 8, dtype=np.uint8)
    return keys.reshape(-1), vals, voff


@pytest.mark.parametrize("devices", [[0], [0, 0], [0, 0, 0], [0] * 4, [0] * 8, [0] * 16], ids=lambda d: f"x{len(d)}")
def test_sharded_vs_single(devices):
    from khipu_amd.trie import trie_root, trie_root_sharded
    from khipu_amd._lib import KhStats
    keys, vals, voff = _rand(200_000, 3)
    exp = trie_root(keys, (vals, voff), klen=32)
    st = KhStats()
    assert trie_root_sharded(keys, (vals, voff), devices, klen=32, stats=st) == exp
    assert st.n_leaves == 200_000 and st.n_inputs == 200_000


def test_sharded_genesis_hash_keys():
    import __graft_entry__ as g
    from khipu_amd.trie import trie_root_sharded
    addrs, vals = g._genesis_inputs()
    for dv in ([0], [0] * 8):
        assert trie_root_sharded(addrs, vals, dv, hash_keys=True).hex() == GENESIS_ROOT


def test_sharded_later_put_wins_across_slices(oracle):
    """A key put in an early slice and again in a later one: the later value wins (slices
    are contiguous and received source-major)."""
    from khipu_amd.trie import trie_root_sharded
    r = random.Random(5)
    base = [bytes(r.getrandbits(8) for _ in range(32)) for _ in range(600)]
    keys = base + base[:200] + base[100:150]
    vals = [bytes([i % 251 + 1]) * (1 + i % 70) for i in range(len(keys))]
    exp = oracle.batch_root(keys, vals, klen=32, nthreads=2)
    for dv in ([0], [0] * 4, [0] * 7):
        assert trie_root_sharded(keys, vals, dv) == exp, len(dv)


def test_sharded_single_nibble_and_empty(oracle):
    """All keys under one top nibble (the root is not a branch: its owner rebuilds from
    depth 0), a single key, and no keys."""
    from khipu_amd.trie import trie_root, trie_root_sharded
    keys, vals, voff = _rand(5000, 9, top=0xB)
    exp = trie_root(keys, (vals, voff), klen=32)
    for dv in ([0], [0] * 8):
        assert trie_root_sharded(keys, (vals, voff), dv, klen=32) == exp
    k1 = [bytes(range(32))]
    v1 = [b"\x01\x02"]
    assert trie_root_sharded(k1, v1, [0] * 4) == oracle.seq_root(k1, v1)
    assert trie_root_sharded([], [], [0, 0]) == EMPTY


def test_sharded_rejects_bad_args():
    from khipu_amd.trie import trie_root_sharded
    from khipu_amd._lib import KhError
    with pytest.raises(KhError):
        trie_root_sharded([bytes(32)], [b"x"], [])
    with pytest.raises(KhError):
        trie_root_sharded([bytes(32)], [b"x"], [7])  # no such device on a 1-GPU box


@pytest.mark.parametrize("devices", [[0], [0, 0, 0], [0] * 8, [0] * 16], ids=lambda d: f"x{len(d)}")
def test_segmented_sharded_vs_cpu_batch(oracle, devices):
    """kh_trie_roots_segmented_sharded (configs[3] across GPUs, SURVEY §8e "Other configs"):
    storage tries split into slot-balanced trie ranges, one per device; every root against
    the CPU batch builder, including empty tries and ranges of a single huge trie."""
    from khipu_amd.trie import trie_roots
    r = random.Random(len(devices))
    tries = []
    for t in range(300):
        n = 0 if t % 37 == 0 else (3000 if t == 150 else r.randrange(1, 60))
        ks = [bytes(r.getrandbits(8) for _ in range(20)) for _ in range(n)]
        vs = [bytes([r.randrange(1, 256)]) * r.randrange(1, 33) for _ in range(n)]
        tries.append((ks, vs))
    got = trie_roots(tries, hash_keys=True, devices=devices)
    assert got == trie_roots(tries, hash_keys=True)
    keys = [k for ks, _ in tries for k in ks]
    vals = [v for _, vs in tries for v in vs]
    so = np.cumsum([0] + [len(ks) for ks, _ in tries]).astype(np.uint64)
    cpu, _ = oracle.batch_roots(keys, vals, klen=20, seg_off=so, hash_keys=True)
    assert got == cpu
    # more devices than tries
    few = tries[:3]
    assert trie_roots(few, hash_keys=True, devices=devices) == trie_roots(few, hash_keys=True)


def test_synth_storage_tries_vs_cpu(oracle):
    """kh_dev_synth_storage (csrc/synth.h configs[3] generator): a range of tries generated on
    the device equals the same tries cut out of a larger range (per-trie determinism), and
    their segmented GPU roots equal the CPU batch builder's on the generated bytes."""
    from khipu_amd.device import Ctx
    ctx = Ctx(0)
    so, keys, vals, voff, seg = ctx.synth_storage(4, 0, 400)
    so2, keys2, vals2, voff2, seg2 = ctx.synth_storage(4, 100, 50)
    a, b = int(so[100]), int(so[150])
    assert int(so2[-1]) == b - a
    assert bytes(keys[32 * a:32 * b].cpu().numpy()) == bytes(keys2[:32 * (b - a)].cpu().numpy())
    v0, v1 = int(voff[a]), int(voff[b])
    assert bytes(vals[v0:v1].cpu().numpy()) == bytes(vals2[:v1 - v0].cpu().numpy())
    counts = np.diff(so.cpu().numpy())
    assert counts.min() >= 1 and counts.max() <= 10_000
    n = int(so[-1])
    hh, ll, _, st = ctx.build(keys, 32, vals, voff, n, seg=seg, nseg=400, hash_keys=True)
    gpu = [hh[s].tobytes() for s in range(400)]
    vo = voff.cpu().numpy().astype(np.uint64)
    cpu, _ = oracle.batch_roots(keys[:32 * n].cpu().numpy(), (vals[:int(vo[-1])].cpu().numpy(), vo), klen=32,
                                seg_off=so.cpu().numpy().astype(np.uint64), hash_keys=True)
    assert gpu == cpu
    # 1-byte values < 0x80 (raw, inline leaves) occur
    lens = np.diff(vo)
    assert (lens == 1).any() and (lens > 1).any()
