"""Multi-process (world_size 2, gloo, CPU) coverage of the sharded state-root driver
(khipu_amd/sharded.py): routing by top-nibble owner, the uneven all-to-all, the
16-reference gather and the host fold — with a CPU backend (host replay of the
device code) standing in for libkhst on each rank.  The GPU backend runs the
same functions with RCCL on the MI355X box (bench.py --gpus N)."""
import os
import random
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


class CpuBackend:
    def __init__(self):
        from tests.emu import emu
        self.emu = emu
        self.last_stats = None
        self.overlap = True  # exercise the asynchronous value exchange (gloo works)

    def empty(self, nbytes, dtype=torch.uint8):
        return torch.empty(nbytes, dtype=dtype)

    def hash_keys(self, addr, n, klen=20):
        a = addr.numpy()
        out = torch.zeros(n * 32 + 64, dtype=torch.uint8)
        for i in range(n):
            out[32 * i:32 * i + 32] = torch.from_numpy(
                np.frombuffer(self.emu.kec256(a[klen * i:klen * i + klen].tobytes()), np.uint8).copy())
        return out

    def hash_partition(self, addr, vals, voff, n, nparts, klen=20):
        """GpuBackend.hash_partition's outputs: the two calls in turn"""
        return self.partition(self.hash_keys(addr, n, klen), vals, voff, n, nparts)

    def partition(self, keys32, vals, voff, n, nparts):
        k = keys32[:n * 32].numpy().reshape(n, 32)
        vo = voff.numpy()
        v = vals.numpy()
        owner = ((k[:, 0] >> 4).astype(np.int64) * nparts) >> 4
        order = np.argsort(owner, kind="stable")
        pk = np.ascontiguousarray(k[order]).reshape(-1)
        lens = (vo[1:] - vo[:-1])[order]
        pv = np.concatenate([v[vo[i]:vo[i + 1]] for i in order] + [np.zeros(0, np.uint8)])
        self.vals_done = self.event()  # exchange() waits on it before the value all-to-all
        cnt = np.bincount(owner, minlength=nparts).astype(np.int64)
        nb = np.bincount(owner, weights=vo[1:] - vo[:-1], minlength=nparts).astype(np.int64)
        return (torch.from_numpy(np.concatenate([pk, np.zeros(64, np.uint8)])),
                torch.from_numpy(np.concatenate([pv, np.zeros(64, np.uint8)])),
                torch.from_numpy(lens.astype(np.int64)), cnt, nb)

    def wait(self, ev):
        pass

    def event(self):
        class Done:
            def synchronize(self):
                pass
        return Done()

    def build(self, keys32, vals, voff, m, depth0, vals_ready=None):
        k = keys32[:m * 32].numpy().reshape(m, 32)
        vo = voff.numpy()
        v = vals.numpy()
        keys = [k[i].tobytes() for i in range(m)]
        vs = [v[vo[i]:vo[i + 1]].tobytes() for i in range(m)]
        res, _ = self.emu.build(keys, vs, depth0=depth0)
        hh = np.frombuffer(b"".join(x[0] for x in res), np.uint8).reshape(len(res), 32).copy()
        ll = np.array([x[1] for x in res], np.uint32)
        ii = np.frombuffer(b"".join(x[2].ljust(32, b"\0") for x in res), np.uint8).reshape(len(res), 32).copy()
        return hh, ll, ii

    def fold(self, hh, ll, ii):
        out = np.zeros(32, np.uint8)
        hh = np.ascontiguousarray(hh, np.uint8)
        ll = np.ascontiguousarray(ll, np.uint32)
        ii = np.ascontiguousarray(ii, np.uint8)
        self.emu.lib().emu_fold16(hh.ctypes.data, ll.ctypes.data, ii.ctypes.data, out.ctypes.data)
        return out.tobytes()

    def sync(self):
        pass


def _records(seed, n, same_top_nibble=False, dup_from=None):
    r = random.Random(seed)
    addrs = [bytes(r.getrandbits(8) for _ in range(20)) for _ in range(n)]
    if dup_from:
        addrs[:len(dup_from)] = dup_from
    from khipu_amd import codec
    vals = [codec.account_rlp(r.randrange(1000), r.randrange(10 ** 20)) for _ in range(n)]
    return addrs, vals


def _worker(rank, world, port, case, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import sys
    sys.path.insert(0, ROOT)
    from khipu_amd import sharded
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        addrs, vals, prehashed = case[:3]
        if len(case) > 3:
            sharded.A2A_CHUNK = case[3]  # force multi-round exchanges
        n_all = len(addrs)
        lo, hi = n_all * rank // world, n_all * (rank + 1) // world
        mine_a, mine_v = addrs[lo:hi], vals[lo:hi]
        klen = 32 if prehashed else 20
        a = torch.from_numpy(np.frombuffer(b"".join(mine_a) + b"\0" * 64, np.uint8).copy())
        v = torch.from_numpy(np.frombuffer(b"".join(mine_v) + b"\0" * 64, np.uint8).copy())
        off = torch.zeros(len(mine_v) + 1, dtype=torch.int64)
        off[1:] = torch.tensor(np.cumsum([len(x) for x in mine_v]), dtype=torch.int64)
        be = CpuBackend()
        root = sharded.sharded_root(be, a, v, off, hi - lo, klen=klen, keys_prehashed=prehashed)
        q.put((rank, root))
    finally:
        dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(case, world=2):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, case, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = [q.get(timeout=240) for _ in procs]
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    roots = {r: x for r, x in out}
    assert len(set(roots.values())) == 1
    return roots[0]


@pytest.mark.parametrize("world", [1, 2, 3, 4, 8])
def test_sharded_root_matches_oracle(oracle, world):
    addrs, vals = _records(1, 600)
    root = _run((addrs, vals, False), world)
    assert root == oracle.seq_root([oracle.kec256(a) for a in addrs], vals)


def test_sharded_duplicates_later_rank_wins(oracle):
    addrs, vals = _records(2, 300)
    addrs[250:260] = addrs[10:20]  # rank 1 re-puts keys first put by rank 0
    root = _run((addrs, vals, False))
    assert root == oracle.seq_root([oracle.kec256(a) for a in addrs], vals)


def test_sharded_single_top_nibble_fallback(oracle):
    """All keys under one top nibble: the root is an extension, not a branch."""
    r = random.Random(3)
    keys = [bytes([0x50 | r.randrange(16)]) + bytes(r.getrandbits(8) for _ in range(31)) for _ in range(100)]
    from khipu_amd import codec
    vals = [codec.storage_value_rlp(r.randrange(1, 1 << 30)) for _ in keys]
    root = _run((keys, vals, True))
    assert root == oracle.seq_root(keys, vals)


def test_sharded_chunked_exchange(oracle):
    """All-to-all split into rounds (the >2 GiB path), forced with a 100-byte chunk."""
    addrs, vals = _records(4, 200)
    root = _run((addrs, vals, False, 100), 3)
    assert root == oracle.seq_root([oracle.kec256(a) for a in addrs], vals)
