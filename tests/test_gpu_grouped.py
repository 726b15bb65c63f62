"""GPU parity of the grouped build (khst.hip grouped_build: large plain roots pipelined over
top-nibble groups on one GPU) against the CPU batch builder (oracle/batch_root.cc, proven
equal to the khipu-faithful oracle in tests/test_batch_root.py), at sizes past its 8M-input
threshold: random keys with repeated puts (later puts win), groups left empty, every key
under one top nibble and long runs of equal 32-bit prefixes (both redone as one plain build),
and synthetic accounts with their addresses hashed on the device."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

N = 9_000_000  # past GROUP_MIN_N (8M)


@pytest.fixture(autouse=True, params=[4, 2])
def groups(request, monkeypatch):
    """The grouped build is a measurement mode (KHST_GROUPS, read per call by the library)."""
    monkeypatch.setenv("KHST_GROUPS", str(request.param))
    return request.param


def _dev(x):
    import torch
    return torch.from_numpy(np.ascontiguousarray(x)).to("cuda:0")


def _values(rng, n):
    """RLP strings of 1..40 random bytes (1-byte values below 0x80 raw), packed."""
    ln = rng.integers(1, 41, n)
    first = rng.integers(1, 256, n).astype(np.uint8)
    raw = (ln == 1) & (first < 0x80)
    enc = np.where(raw, 1, ln + 1)
    off = np.zeros(n + 1, np.uint64)
    off[1:] = np.cumsum(enc)
    vb = rng.integers(0, 256, int(off[-1]) + 64, dtype=np.uint8)
    st = off[:-1].astype(np.int64)
    vb[st[~raw]] = (0x80 + ln[~raw]).astype(np.uint8)
    vb[st[~raw] + 1] = first[~raw]
    vb[st[raw]] = first[raw]
    return vb, off


def _check(ctx, oracle, keys, vb, off):
    n = len(off) - 1
    hh, ll, _, st = ctx.build(_dev(keys.reshape(-1)), 32, _dev(vb), _dev(off.astype(np.int64)), n)
    cpu, cst = oracle.batch_roots(keys.reshape(-1), (vb, off), klen=32)
    assert hh[0].tobytes() == cpu[0]
    assert st.n_leaves == cst["distinct"] and st.n_node_hashes == cst["node_hashes"]
    return st


def _grouped(st, groups):
    assert st.n_groups == groups, st.n_groups


def test_grouped_random_with_repeats(khst, oracle, groups):
    from khipu_amd.device import Ctx
    rng = np.random.default_rng(41)
    keys = rng.integers(0, 256, (N, 32), dtype=np.uint8)
    dup = rng.choice(N, N // 20, replace=False)
    keys[dup] = keys[rng.choice(N, N // 20, replace=False)]  # 5% of the puts repeat a key
    vb, off = _values(rng, N)
    _grouped(_check(Ctx(0), oracle, keys, vb, off), groups)


def test_grouped_empty_groups_and_one_nibble(khst, oracle, groups):
    """Keys under top nibbles 0 and 1 only (groups 1..3 empty); then every key under nibble 5
    (the root is not a branch: one plain build)."""
    from khipu_amd.device import Ctx
    rng = np.random.default_rng(42)
    ctx = Ctx(0)
    keys = rng.integers(0, 256, (N, 32), dtype=np.uint8)
    keys[:, 0] &= 0x1F
    vb, off = _values(rng, N)
    _grouped(_check(ctx, oracle, keys, vb, off), groups)
    keys[:, 0] = 0x50 | (keys[:, 0] & 0x0F)
    assert _check(ctx, oracle, keys, vb, off).n_groups == 0  # one plain build


def test_grouped_long_prefix_runs(khst, oracle, groups):
    """Runs of 200 keys sharing their first 32 bits (longer than the tie kernel's runs): the
    grouped build hands over to one plain build with the full 256-bit sort."""
    from khipu_amd.device import Ctx
    rng = np.random.default_rng(43)
    keys = rng.integers(0, 256, (N, 32), dtype=np.uint8)
    keys[1000:1200, :4] = keys[1000, :4]
    keys[5_000_000:5_000_200, :4] = keys[5_000_000, :4]
    vb, off = _values(rng, N)
    assert _check(Ctx(0), oracle, keys, vb, off).n_groups == 0  # one plain build


def test_grouped_synthetic_accounts(khst, oracle, groups):
    """configs[1]-style accounts at 10M, addresses hashed on the device (KH_HASH_KEYS)."""
    import torch
    from khipu_amd.device import Ctx
    ctx = Ctx(0)
    n = 10_000_000
    addr, vals, voff = ctx.synth_accounts(4, 0, n)
    hh, _, _, st = ctx.build(addr, 20, vals, voff, n, hash_keys=True)
    torch.cuda.synchronize()
    a = addr[:20 * n].cpu().numpy()
    vo = voff.cpu().numpy().astype(np.uint64)
    vb = vals[:int(vo[-1])].cpu().numpy()
    cpu, cst = oracle.batch_roots(a, (vb, vo), klen=20, hash_keys=True)
    assert hh[0].tobytes() == cpu[0]
    assert st.n_node_hashes == cst["node_hashes"] and st.n_key_perms == n
    _grouped(st, groups)
