"""The torch sharded driver (khipu_amd/sharded.py, what `bench.py --gpus N` runs) at world
sizes 2, 4 and 8 with the REAL device library on every rank: each rank is a process on
the box's one GPU running GpuBackend (k_hash_keys, kh_dev_partition_ev with the value
copy still in flight, owner-shaped shard builds from depth 1, the host fold), and the
collectives are staged through host memory over gloo, since RCCL refuses two ranks on
one device.  Only the transport differs from the N-GPU run: the partition, the
exchange's ordering (key all-to-all first, value all-to-all after the partition's
event, the build waiting on vals_ready) and the owner layout (two nibbles per rank at
world 8) are the ones the 8-GPU node runs.

Parity: rank 0 compares the sharded root with a single-GPU build of the same synthetic
workload (sharded.self_check) and with the CPU batch builder (oracle/batch_root.cc)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
N_ACCOUNTS = 400_000


class _Done:
    def wait(self):
        pass


class HostStagedDist:
    """torch.distributed with every collective of sharded.py run on host copies of the
    device tensors (gloo); everything else is passed through."""

    def __getattr__(self, k):
        return getattr(dist, k)

    @staticmethod
    def all_to_all_single(out, inp, out_splits=None, in_splits=None, async_op=False):
        o = torch.empty(out.shape, dtype=out.dtype)
        dist.all_to_all_single(o, inp.cpu(), out_splits, in_splits)
        out.copy_(o)
        return _Done() if async_op else None

    @staticmethod
    def all_reduce(t, op=dist.ReduceOp.SUM):
        c = t.cpu()
        dist.all_reduce(c, op=op)
        t.copy_(c)

    @staticmethod
    def all_gather_into_tensor(out, inp):
        parts = [torch.empty(inp.shape, dtype=inp.dtype) for _ in range(dist.get_world_size())]
        dist.all_gather(parts, inp.cpu())
        out.copy_(torch.cat(parts))

    @staticmethod
    def broadcast(t, src):
        c = t.cpu()
        dist.broadcast(c, src)
        t.copy_(c)


def _worker(rank, world, port, n_total, chunk, q, cpu=True):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import sys
    sys.path.insert(0, ROOT)
    from khipu_amd import sharded
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        sharded.dist = HostStagedDist()
        if chunk:
            sharded.A2A_CHUNK = chunk  # multi-round exchanges (the > 1 GiB-per-peer path)
        torch.cuda.set_device(0)
        be = sharded.GpuBackend(0)
        first = n_total * rank // world
        n = n_total * (rank + 1) // world - first
        addr, vals, voff = be.ctx.synth_accounts(5, first, n)
        be.sync()
        roots = [sharded.sharded_root(be, addr, vals, voff, n) for _ in range(2)]  # workspaces reused
        be.sync()
        out = {"rank": rank, "roots": [r.hex() for r in roots], "leaves": int(be.last_stats.n_leaves)}
        if rank == 0:
            ok, rep = sharded.self_check(be, 5, n_total, roots[-1])
            out["self_check"] = ok
            out["single"] = rep["single_gpu_root"]
        if rank == 0 and cpu:
            from oracle import oracle as O
            a, v, o = be.ctx.synth_accounts(5, 0, n_total)
            a, v, o = a.cpu().numpy(), v.cpu().numpy(), o.cpu().numpy()
            out["cpu"] = O.batch_root(a[:20 * n_total], (v, o[:n_total + 1]), klen=20, hash_keys=True).hex()
        q.put(out)
    except BaseException as e:  # reported to the parent, which fails the test
        q.put({"rank": rank, "error": repr(e)})
        raise
    finally:
        dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.gpu
@pytest.mark.parametrize("world,chunk", [(2, 0), (4, 0), (8, 0), (3, 1 << 16)])
def test_sharded_torch_world(world, chunk):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, N_ACCOUNTS, chunk, q)) for r in range(world)]
    for p in procs:
        p.start()
    try:
        outs = [q.get(timeout=90) for _ in procs]
    finally:
        for p in procs:
            p.join(30)
            if p.exitcode is None:
                p.kill()
    errs = [o for o in outs if "error" in o]
    assert not errs, errs
    for p in procs:
        assert p.exitcode == 0
    r0 = next(o for o in outs if o["rank"] == 0)
    roots = {r for o in outs for r in o["roots"]}
    assert roots == {r0["cpu"]}, (roots, r0["cpu"])
    assert r0["self_check"] and r0["single"] == r0["cpu"]
    # every rank built its owner shard: the leaves add up to the workload
    assert sum(o["leaves"] for o in outs) == N_ACCOUNTS
