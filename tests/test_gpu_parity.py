"""GPU parity: libkhst.so's HIP path vs the oracle (bit-exact; integer/byte work).

Every test calls through the C ABI (ctypes) and compares against
oracle/khipu_oracle.cc (khipu-faithful sequential trie) on the same inputs, or
against the pinned in-tree known answers.  At full size (1M accounts) parity is
checked against the oracle directly plus size-independent properties
(input-order invariance, determinism, sharded == single-device root).
"""
import os
import random

import numpy as np
import pytest

from tests import cases as C

pytestmark = pytest.mark.gpu

GENESIS_ROOT = "d7f8974fb5ac78d9ac099b9ad5018bedc2ce0a72dad1827a1709da30580f0544"


def test_kec256_known_answers(khst):
    # Account.scala:13-17, BlockHeader.scala:14
    got = khst.kec256_batch([b"", b"\x80", b"\xc0"])
    assert got[0].hex() == "c5d2460186f7233c927e7db2dcc703c0e500b653ca82273b7bfad8045d85a470"
    assert got[1].hex() == "56e81f171bcc55a6ff8345e692c0f86e5b48e01b996cadc001622fb5e363b421"
    assert got[2].hex() == "1dcc4de8dec75d7aab85b567b6ccd41ad312451b948a7413f0a142fd40d49347"


def test_kec256_batch_vs_oracle(khst, oracle):
    r = random.Random(3)
    lens = list(range(0, 300)) + [407, 408, 409, 543, 544, 545, 600, 1000, 4096]
    msgs = [bytes(r.getrandbits(8) for _ in range(L)) for L in lens]
    # odd offsets: messages packed back to back at arbitrary alignment
    got = khst.kec256_batch(msgs)
    for m, h in zip(msgs, got):
        assert h == oracle.kec256(m), len(m)


@pytest.mark.parametrize("case", C.all_cases(), ids=lambda c: c[0])
def test_trie_root_vs_oracle(khst, oracle, case):
    name, keys, vals = case
    st = khst.KhStats()
    got = khst.trie_root(keys, vals, stats=st)
    assert got == oracle.seq_root(keys, vals), name
    if name in ("prefix_ties", "prefix_ties_long"):  # a 64-run is fixed locally, a 150-run is not
        assert st.full_sort == (1 if name == "prefix_ties_long" else 0), name


def test_trie_root_hash_keys(khst, oracle):
    r = random.Random(9)
    addrs = [bytes(r.getrandbits(8) for _ in range(20)) for _ in range(2000)]
    vals = [C.account_value(r) for _ in addrs]
    got = khst.trie_root(addrs, vals, hash_keys=True)
    assert got == oracle.seq_root([oracle.kec256(a) for a in addrs], vals)


def test_empty_trie(khst):
    assert khst.trie_root([], []) == khst.EMPTY_TRIE_HASH


def test_genesis_state_root(khst):
    import __graft_entry__ as g
    addrs, vals = g._genesis_inputs()
    st = khst.KhStats()
    assert khst.trie_root(addrs, vals, hash_keys=True, stats=st).hex() == GENESIS_ROOT
    assert st.n_leaves == 8893


def test_segmented_vs_oracle(khst, oracle):
    tries = C.segmented_case()
    got = khst.trie_roots(tries)
    for (ks, vs), g in zip(tries, got):
        exp = oracle.seq_root(ks, vs) if ks else khst.EMPTY_TRIE_HASH
        assert g == exp


def test_write_back_node_set(khst, oracle):
    """Emitted (hash -> RLP) == every node reachable from the oracle's root with
    encoding >= 32 B plus the root (MerklePatriciaTrie.scala:505-511)."""
    for name, keys, vals in C.all_cases(big=False):
        if name in ("duplicates", "prefix_ties_dups", "prefix_ties_long"):
            continue
        root, nodes = khst.trie_root_nodes(keys, vals)
        t = oracle.Trie()
        for k, v in zip(keys, vals):
            t.put(k, v)
        assert root == t.root_hash(), name
        exp = t.reachable()
        assert nodes == exp, name
        # every emitted node is also an Updated entry of the faithful log
        upd = t.updated()
        assert all(h in upd and upd[h] == e for h, e in nodes.items()), name


def test_mirror_api(khst, oracle):
    r = random.Random(4)
    t = khst.MerklePatriciaTrie()
    o = oracle.Trie()
    keys = [bytes(r.getrandbits(8) for _ in range(32)) for _ in range(500)]
    for k in keys:
        v = C.storage_value(r)
        t.put(k, v)
        o.put(k, v)
    assert t.root_hash() == o.root_hash()
    for k in keys[:200]:
        t.remove(k)
        o.remove(k)
    assert t.root_hash() == o.root_hash()
    assert t.get(keys[300]) == o.get(keys[300])
    assert t.get(keys[0]) is None


def test_synth_generator_matches_host_replay(khst):
    from khipu_amd.device import Ctx
    from tests.emu import emu
    ctx = Ctx(0)
    n = 5000
    addr, vals, voff = ctx.synth_accounts(2, 1234, n)
    ea, ev, eo = emu.synth(2, 1234, n)
    vo = voff.cpu().numpy().astype(np.uint64)
    assert np.array_equal(vo, eo)
    assert np.array_equal(addr[:20 * n].cpu().numpy(), ea.reshape(-1))
    assert np.array_equal(vals[:int(vo[n])].cpu().numpy(), ev)


def _device_synth_root(ctx, n, cfg=1, depth0=0):
    addr, vals, voff = ctx.synth_accounts(cfg, 0, n)
    return ctx.build(addr, 20, vals, voff, n, depth0=depth0, hash_keys=True), (addr, vals, voff)


def test_synth_100k_vs_oracle(khst, oracle):
    from khipu_amd.device import Ctx
    ctx = Ctx(0)
    n = 100_000
    (hh, ll, ii, st), (addr, vals, voff) = _device_synth_root(ctx, n)
    a = addr[:20 * n].cpu().numpy().reshape(n, 20)
    keys = np.frombuffer(b"".join(oracle.kec256(x.tobytes()) for x in a), np.uint8)
    vo = voff.cpu().numpy().astype(np.uint64)
    vb = vals[:int(vo[n])].cpu().numpy()
    assert hh[0].tobytes() == oracle.seq_root_packed(keys, 32, vb, vo, n)
    assert st.n_leaves == n and st.n_key_perms == n


def test_sharded_fold_equals_single(khst, oracle):
    """16 top-nibble subtries (the multi-GPU shard unit) folded on the host == single build."""
    from khipu_amd.device import Ctx, fold_root16
    ctx = Ctx(0)
    for n in (3, 40, 20_000):
        (h0, l0, i0, _), bufs = _device_synth_root(ctx, n, cfg=4)
        hh, ll, ii, _ = ctx.build(bufs[0], 20, bufs[1], bufs[2], n, depth0=1, hash_keys=True)
        if (ll > 0).sum() >= 2:
            assert fold_root16(hh, ll, ii) == h0[0].tobytes(), n


def test_full_size_1m(khst, oracle):
    """configs[1] size: 1M synthetic accounts — oracle parity, determinism, order invariance."""
    from khipu_amd.device import Ctx
    ctx = Ctx(0)
    n = 1_000_000
    (hh, ll, ii, st), (addr, vals, voff) = _device_synth_root(ctx, n)
    root = hh[0].tobytes()
    # determinism
    hh2, _, _, _ = ctx.build(addr, 20, vals, voff, n, hash_keys=True)
    assert hh2[0].tobytes() == root
    # oracle (khipu-faithful sequential puts)
    a = addr[:20 * n].cpu().numpy().reshape(n, 20)
    keys = np.frombuffer(b"".join(oracle.kec256(x.tobytes()) for x in a), np.uint8)
    vo = voff.cpu().numpy().astype(np.uint64)
    vb = vals[:int(vo[n])].cpu().numpy()
    assert root == oracle.seq_root_packed(keys, 32, vb, vo, n)
    # the independent all-core batch builder (the full-size check bench.py uses at 100M)
    roots, bst = oracle.batch_roots(a.reshape(-1), (vb, vo), klen=20, hash_keys=True)
    assert roots[0] == root
    assert (bst["leaves"], bst["node_hashes"], bst["node_perms"]) == (st.n_leaves, st.n_node_hashes, st.n_node_perms)
    # input-order invariance: the same puts in reverse order give the same root
    lens = np.diff(vo)[::-1].astype(np.int64)
    new_off = np.zeros(n + 1, np.uint64)
    new_off[1:] = np.cumsum(lens)
    src = vo[:-1][::-1].astype(np.int64)
    total = int(new_off[n])
    gather = np.repeat(src - new_off[:-1].astype(np.int64), lens) + np.arange(total)
    rv = vb[gather]
    rk = np.ascontiguousarray(keys.reshape(n, 32)[::-1]).reshape(-1)
    assert khst.trie_root(rk, (rv, new_off), klen=32) == root


def test_sharded_driver_rccl_world1(khst, oracle):
    """khipu_amd/sharded.py over RCCL (world size 1 on this box; the routing logic at
    world sizes 2 and 3 is covered with gloo in tests/test_multigpu.py)."""
    import socket
    import torch
    import torch.distributed as dist
    from khipu_amd import sharded
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1,
                            device_id=torch.device("cuda:0"))
    try:
        be = sharded.GpuBackend(0)
        n = 50_000
        addr, vals, voff = be.ctx.synth_accounts(7, 0, n)
        root = sharded.sharded_root(be, addr, vals, voff, n)
        hh, _, _, _ = be.ctx.build(addr, 20, vals, voff, n, hash_keys=True)
        assert root == hh[0].tobytes()
    finally:
        dist.destroy_process_group()


def test_build_waits_for_late_values(khst, oracle):
    """kh_dev_trie_build_ev (the multi-GPU exchange's overlap): the values and offsets land
    on another stream after a delay; the build sorts and derives the topology meanwhile
    and reads them only after the event.  Without the wait it would hash zero bytes."""
    import torch
    from khipu_amd.device import Ctx
    ctx = Ctx(0)
    for n in (5_000, 300_000):
        (h0, _, _, _), (addr, vals, voff) = _device_synth_root(ctx, n, cfg=3)
        keys = torch.empty(n * 32 + 64, dtype=torch.uint8, device="cuda:0")
        ctx.build(addr, 20, vals, voff, n, hash_keys=True)  # warm the workspace
        from khipu_amd._lib import check, lib
        from khipu_amd.device import _ptr
        check(lib().kh_dev_hash_keys(ctx.h, _ptr(addr), 20, n, _ptr(keys)))
        torch.cuda.synchronize()
        late_v = torch.zeros_like(vals)
        late_o = torch.zeros_like(voff)
        side = torch.cuda.Stream()
        with torch.cuda.stream(side):
            torch.cuda._sleep(50_000_000)  # ~20 ms of spinning before the copies
            late_v.copy_(vals)
            late_o.copy_(voff)
            ev = torch.cuda.Event()
            ev.record()
        hh, _, _, _ = ctx.build(keys, 32, late_v, late_o, n, depth0=0, vals_ready=ev)
        assert hh[0].tobytes() == h0[0].tobytes(), n
        torch.cuda.synchronize()


@pytest.mark.parametrize("koff,voff_shift", [(8, 0), (1, 3), (0, 5)])
def test_device_build_misaligned_buffers(khst, oracle, koff, voff_shift):
    """Device keys / values at arbitrary byte offsets (the ABI takes plain pointers):
    keys not 16-byte aligned are copied into the workspace; value spans are staged
    by aligned words whatever the base alignment."""
    import torch
    from khipu_amd.device import Ctx
    ctx = Ctx(0)
    r = random.Random(17 + koff)
    keys = [bytes(r.getrandbits(8) for _ in range(32)) for _ in range(3000)]
    vals = [C.account_value(r) if i % 3 else C.storage_value(r) for i in range(len(keys))]
    kb = torch.zeros(len(keys) * 32 + 64, dtype=torch.uint8)
    kb[koff:koff + 32 * len(keys)] = torch.frombuffer(bytearray(b"".join(keys)), dtype=torch.uint8)
    blob = b"".join(vals)
    vb = torch.zeros(len(blob) + 64, dtype=torch.uint8)
    vb[voff_shift:voff_shift + len(blob)] = torch.frombuffer(bytearray(blob), dtype=torch.uint8)
    off = torch.tensor(np.concatenate([[0], np.cumsum([len(v) for v in vals])]), dtype=torch.int64)
    dk, dv, do = kb.cuda()[koff:], vb.cuda()[voff_shift:], off.cuda()
    hh, _, _, _ = ctx.build(dk, 32, dv, do, len(keys))
    assert hh[0].tobytes() == oracle.seq_root(keys, vals)


@pytest.mark.parametrize("nparts", [1, 2, 3, 8, 16])
def test_partition_vs_host(khst, nparts):
    """kh_dev_partition (grouped span copy) == a stable numpy partition by top-nibble owner:
    keys, value bytes, value lengths, per-owner counts and bytes; ragged 0..300-byte values
    at unaligned offsets, plus the empty batch.  Both the synchronous copy and the deferred
    one (kh_dev_partition_ev: the values checked after the current stream waits on
    vals_done, as exchange() orders the value all-to-all)."""
    import torch
    from khipu_amd import sharded
    rng = np.random.default_rng(nparts)
    be = sharded.GpuBackend(0)
    for overlap, n in [(o, n) for o in (True, False) for n in (0, 1, 777, 100_003)]:
        be.overlap = overlap
        lens = rng.integers(0, 301, n).astype(np.int64)
        short = rng.random(n) < 0.5
        lens[short] = rng.integers(0, 12, int(short.sum()))
        vo = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
        v = rng.integers(0, 256, int(vo[-1]) + 64, dtype=np.uint8)
        k = rng.integers(0, 256, n * 32 + 64, dtype=np.uint8)
        kd, vd, od = (torch.from_numpy(x).to("cuda:0") for x in (k, v, vo))
        pk, pv, pl, cnt, nb = be.partition(kd, vd, od, n, nparts)
        assert (be.vals_done is not None) == overlap
        if overlap:
            be.wait(be.vals_done)
            pv = pv.clone()  # on the current stream, after the wait
        torch.cuda.synchronize()
        kk = k[:n * 32].reshape(n, 32)
        owner = ((kk[:, 0] >> 4).astype(np.int64) * nparts) >> 4
        order = np.argsort(owner, kind="stable")
        assert np.array_equal(cnt, np.bincount(owner, minlength=nparts)[:nparts])
        assert np.array_equal(nb, np.bincount(owner, weights=lens, minlength=nparts)[:nparts].astype(np.int64))
        if n == 0:
            continue
        assert np.array_equal(pk[:n * 32].cpu().numpy(), kk[order].reshape(-1))
        assert np.array_equal(pl[:n].cpu().numpy(), lens[order])
        want = np.concatenate([v[vo[i]:vo[i + 1]] for i in order])
        assert np.array_equal(pv[:len(want)].cpu().numpy(), want)


def test_partition_keys_8byte_aligned(khst):
    """Keys at an 8-byte but not 16-byte aligned address take k_part_place's 8-byte word
    moves (16-byte aligned keys and outputs take the 16-byte ones): same stable partition."""
    import torch
    from khipu_amd import sharded
    rng = np.random.default_rng(7)
    be = sharded.GpuBackend(0)
    be.overlap = False
    n, nparts = 50_001, 8
    lens = rng.integers(0, 90, n).astype(np.int64)
    vo = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    v = rng.integers(0, 256, int(vo[-1]) + 64, dtype=np.uint8)
    k = rng.integers(0, 256, n * 32 + 64, dtype=np.uint8)
    kbuf = torch.zeros(n * 32 + 128, dtype=torch.uint8, device="cuda:0")
    kd = kbuf[8:8 + n * 32 + 64]
    kd.copy_(torch.from_numpy(k))
    assert kd.data_ptr() % 16 == 8
    vd, od = (torch.from_numpy(x).to("cuda:0") for x in (v, vo))
    pk, pv, pl, cnt, nb = be.partition(kd, vd, od, n, nparts)
    torch.cuda.synchronize()
    kk = k[:n * 32].reshape(n, 32)
    owner = ((kk[:, 0] >> 4).astype(np.int64) * nparts) >> 4
    order = np.argsort(owner, kind="stable")
    assert np.array_equal(cnt, np.bincount(owner, minlength=nparts)[:nparts])
    assert np.array_equal(pk[:n * 32].cpu().numpy(), kk[order].reshape(-1))
    assert np.array_equal(pl[:n].cpu().numpy(), lens[order])
    want = np.concatenate([v[vo[i]:vo[i + 1]] for i in order])
    assert np.array_equal(pv[:len(want)].cpu().numpy(), want)


@pytest.mark.parametrize("nparts", [2, 8, 16])
def test_hash_partition_vs_host(khst, oracle, nparts):
    """kh_dev_hash_partition_ev (the keys kec256'd in a pass that writes each owner byte) ==
    the oracle's kec256 of every address, partitioned stably by top-nibble owner: keys,
    lengths, value bytes, counts and bytes per owner; 20-byte addresses (the short
    single-block hash), 200-byte keys (multi-block), n not a multiple of the 2,048-record
    tile nor of the count pass's 8 owner bytes per thread (1, 7, 2,049), and the empty batch."""
    import torch
    from khipu_amd import sharded
    rng = np.random.default_rng(100 + nparts)
    be = sharded.GpuBackend(0)
    for klen, n in ((20, 0), (20, 1), (20, 7), (20, 2_049), (20, 5_000), (20, 70_001), (200, 3_001)):
        lens = rng.integers(0, 120, n).astype(np.int64)
        vo = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
        v = rng.integers(0, 256, int(vo[-1]) + 64, dtype=np.uint8)
        a = rng.integers(0, 256, n * klen + 64, dtype=np.uint8)
        ad, vd, od = (torch.from_numpy(x).to("cuda:0") for x in (a, v, vo))
        pk, pv, pl, cnt, nb = be.hash_partition(ad, vd, od, n, nparts, klen)
        be.wait(be.vals_done)
        pv = pv.clone()
        torch.cuda.synchronize()
        kk = np.frombuffer(b"".join(oracle.kec256(a[klen * i:klen * i + klen].tobytes()) for i in range(n)),
                           np.uint8).reshape(n, 32)
        owner = ((kk[:, 0] >> 4).astype(np.int64) * nparts) >> 4
        order = np.argsort(owner, kind="stable")
        assert np.array_equal(cnt, np.bincount(owner, minlength=nparts)[:nparts]), (klen, n)
        assert np.array_equal(nb, np.bincount(owner, weights=lens, minlength=nparts)[:nparts].astype(np.int64))
        if n == 0:
            continue
        assert np.array_equal(pk[:n * 32].cpu().numpy(), kk[order].reshape(-1)), (klen, n)
        assert np.array_equal(pl[:n].cpu().numpy(), lens[order])
        want = np.concatenate([v[vo[i]:vo[i + 1]] for i in order])
        assert np.array_equal(pv[:len(want)].cpu().numpy(), want)


def test_branch_levels_vs_oracle(khst, oracle):
    """The N1 branch kernels give the oracle's roots on every edge case, storage tries with
    inline children and segmented builds, and a 200k device build's root and permutation
    count equal the CPU batch builder's."""
    variant = "default"
    for name, keys, vals in C.all_cases(big=False):
        assert khst.trie_root(keys, vals) == oracle.seq_root(keys, vals), (variant, name)
    tries = C.segmented_case()
    for (ks, vs), g in zip(tries, khst.trie_roots(tries)):
        assert g == (oracle.seq_root(ks, vs) if ks else khst.EMPTY_TRIE_HASH), variant
    from khipu_amd.device import Ctx
    ctx = Ctx(0)
    (hh, _, _, st), (addr, vals, voff) = _device_synth_root(ctx, 200_000)
    a = addr[:20 * 200_000].cpu().numpy()
    vo = voff.cpu().numpy().astype(np.uint64)
    roots, bst = oracle.batch_roots(a, (vals[:int(vo[-1])].cpu().numpy(), vo), klen=20, hash_keys=True)
    assert hh[0].tobytes() == roots[0] and st.n_node_perms == bst["node_perms"], variant


def test_radix_tile_thresholds(khst, oracle):
    """The radix sort's tile size changes with n (prims.h radix_items: 1024-key tiles up to
    65,536 keys, 4096 above, 8192 for 32-bit words from 4,194,304 keys): hashed-key builds one
    key either side of both thresholds, with the one-sweep passes' look-back over many tiles;
    roots and node counts equal the CPU batch builder's."""
    from khipu_amd.device import Ctx
    ctx = Ctx(0)
    for n in (65_535, 65_536, 65_537, (1 << 22) - 1, 1 << 22, (1 << 22) + 1):
        (hh, _, _, st), (addr, vals, voff) = _device_synth_root(ctx, n, cfg=5)
        a = addr[:20 * n].cpu().numpy()
        vo = voff[:n + 1].cpu().numpy().astype(np.uint64)
        roots, bst = oracle.batch_roots(a, (vals[:int(vo[-1])].cpu().numpy(), vo), klen=20, hash_keys=True)
        assert hh[0].tobytes() == roots[0], n
        assert (bst["leaves"], bst["node_hashes"]) == (st.n_leaves, st.n_node_hashes), n


def test_tie_runs_across_blocks(khst, oracle):
    """Many runs of equal 32-bit sort prefixes (2..64 keys each, some spanning the tie
    kernel's 1,024-position blocks), raw 32-byte keys: the runs are ordered by the whole
    key and their inner boundaries valued by the tie kernel (k_lcp skips them); with and
    without repeated keys (a dedup shifts positions: k_lcp then values every boundary).
    Roots equal the CPU batch builder's."""
    import random
    r = random.Random(23)
    keys = []
    while len(keys) < 60_000:
        pre = bytes(r.getrandbits(8) for _ in range(4))
        keys += [pre + bytes(r.getrandbits(8) for _ in range(28)) for _ in range(r.randint(2, 64))]
    keys += [bytes(r.getrandbits(8) for _ in range(32)) for _ in range(20_000)]
    r.shuffle(keys)
    vals = [bytes([r.getrandbits(8) | 1]) * r.choice([1, 5, 40, 80]) for _ in keys]
    from khipu_amd._lib import KhStats
    want = oracle.batch_root(keys, vals, nthreads=4)
    st = KhStats()
    assert khst.trie_root(keys, vals, stats=st) == want
    assert st.full_sort == 0
    rep = keys + [keys[r.randrange(len(keys))] for _ in range(500)]
    rvals = vals + [bytes([7]) * 33 for _ in range(500)]
    assert khst.trie_root(rep, rvals) == oracle.batch_root(rep, rvals, nthreads=4)


def test_wide_branches_in_large_levels(khst, oracle):
    """The large levels' child table reaches 4,096 key positions from a branch's first key;
    a wave holding a branch that spans more takes the per-child form (k_branch_fused).  3M
    random raw keys (a 65,536-branch depth-4 level and a ~0.9M-branch depth-5 level) plus
    a 20k-key cluster under one 5-nibble prefix and a 6k-key cluster under one 6-nibble
    prefix, whose ancestors in those levels span 6k-20k keys; the root equals the CPU batch
    builder's."""
    rng = np.random.default_rng(31)
    n = 3_000_000
    keys = rng.integers(0, 256, (n + 26_000, 32), dtype=np.uint8)
    keys[n:n + 20_000, :2] = [0x12, 0x34]
    keys[n:n + 20_000, 2] = (keys[n:n + 20_000, 2] & 0x0F) | 0x50  # prefix 0x1234 5
    keys[n + 20_000:, :3] = [0xAB, 0xCD, 0xEF]                      # prefix 0xABCDEF
    rng.shuffle(keys)
    lens = rng.choice([1, 33, 70, 90], len(keys)).astype(np.uint64)
    off = np.zeros(len(keys) + 1, np.uint64)
    off[1:] = np.cumsum(lens)
    vals = rng.integers(1, 256, int(off[-1]), dtype=np.uint8)
    flat = np.ascontiguousarray(keys).reshape(-1)
    roots, _ = oracle.batch_roots(flat, (vals, off), klen=32)
    assert khst.trie_root(flat, (vals, off), klen=32) == roots[0]


def test_hashed_keys_with_repeats(khst, oracle):
    """Hashed-key builds (the plain path: 32-bit sort prefixes from the hashing pass, ties
    ordered by the whole key, the last put of a repeated key kept) over sizes around the
    radix tile and wave boundaries; roots equal the CPU batch builder's."""
    import random
    r = random.Random(17)
    for n in (2, 3, 17, 255, 256, 257, 1000, 2049, 4099):
        base = [bytes(r.getrandbits(8) for _ in range(20)) for _ in range(n)]
        keys = base + [base[r.randrange(n)] for _ in range(n // 3)]  # repeats anywhere
        r.shuffle(keys)
        vals = [bytes([r.getrandbits(8) | 1]) * r.choice([1, 3, 40, 90]) for _ in keys]
        assert khst.trie_root(keys, vals, hash_keys=True) == oracle.batch_root(keys, vals, klen=20, hash_keys=True,
                                                                                nthreads=2), n


def test_6m_with_repeats(khst, oracle):
    """6M accounts plus 200k repeated addresses with new bodies before and after them,
    against the CPU batch builder (later puts win)."""
    import torch
    from khipu_amd.device import Ctx
    ctx = Ctx(0)
    n = 6_000_000
    addr, vals, voff = ctx.synth_accounts(5, 0, n)
    torch.cuda.synchronize()
    a = addr[:20 * n].cpu().numpy().reshape(n, 20)
    vo = voff.cpu().numpy().astype(np.uint64)
    vb = vals[:int(vo[n])].cpu().numpy()
    rng = np.random.default_rng(8)
    rep = rng.integers(0, n, 200_000)
    rk = a[rep]
    rv = rng.integers(0, 256, 200_000 * 70, dtype=np.uint8)
    keys = np.concatenate([rk[:100_000], a, rk[100_000:]]).reshape(-1)
    vbytes = np.concatenate([rv[:100_000 * 70], vb, rv[100_000 * 70:]])
    lens = np.concatenate([np.full(100_000, 70), np.diff(vo), np.full(100_000, 70)]).astype(np.uint64)
    off = np.zeros(len(lens) + 1, np.uint64)
    off[1:] = np.cumsum(lens)
    d_k = torch.from_numpy(np.ascontiguousarray(keys)).to("cuda:0")
    d_v = torch.from_numpy(np.concatenate([vbytes, np.zeros(64, np.uint8)])).to("cuda:0")
    d_o = torch.from_numpy(off.astype(np.int64)).to("cuda:0")
    N = len(lens)
    hh, _, _, st = ctx.build(d_k, 20, d_v, d_o, N, hash_keys=True)
    roots, bst = oracle.batch_roots(keys, (vbytes, off), klen=20, hash_keys=True)
    assert hh[0].tobytes() == roots[0]
    assert st.n_leaves == bst["leaves"]


@pytest.mark.gpu
def test_lane_spread_keccak_on_device(khst):
    """N1: the lane-spread permutation (keccak_xlane.h, 25 lanes per state in 32-lane groups,
    LDS round trips) == keccak.h's one-thread permutation on 512 random states, 1 and 3
    permutations in a row, run as the real device code (scripts/xlane_check, built by
    __graft_entry__.build()); it also reports the latency per permutation of both forms."""
    import json
    import subprocess
    exe = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "scripts", "xlane_check")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    d = json.loads(r.stdout.strip().splitlines()[-1])
    assert d["equal"] is True
    assert d["us_per_perm"]["xlane_1wave"] < d["us_per_perm"]["thread_1wave"]
