"""BASELINE.json configs[4] at its configured size: the 100M-account synthetic state root
(csrc/synth.h, config 5 -- the bench workload), keys hashed on the device.

- one GPU: the plain build's root against the independent CPU batch builder over all 100M
  accounts (oracle/batch_root.cc, 16 threads) and the pinned root (sharded.PINNED_ROOTS);
- the 8-way owner layout of SURVEY §8e through the C ABI: kh_trie_root_sharded over the
  device list [0]*8 -- eight top-nibble owner shards of ~12.5M records each (two root
  nibbles per shard), built on the box's one GPU through the repeated-device path of
  csrc/sharded.h, the 16 references folded on the host -- must give the same root;
- the torch driver bench.py --gpus 8 runs (khipu_amd/sharded.py) at world 8 with 12.5M
  accounts per rank (tests/test_gpu_sharded_torch.py's host-staged transport).

The reference computes this root by folding MerklePatriciaTrie.put over the accounts
(TrieAccounts.flush, TrieAccounts.scala:22-28 -> MerklePatriciaTrie.scala:157-281, rootHash
:78,169); the batch builder is proven equal to that fold by tests/test_batch_root.py."""
import time

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

N = 100_000_000
CFG = 5


@pytest.mark.timeout(900)
def test_config4_100m_single_and_8_owner_shards(khst, oracle):
    import torch
    from khipu_amd.device import Ctx
    from khipu_amd.sharded import PINNED_ROOTS
    from khipu_amd.trie import trie_root_sharded
    from khipu_amd._lib import KhStats
    ctx = Ctx(0)
    addr, vals, voff = ctx.synth_accounts(CFG, 0, N)
    hh, _, _, st = ctx.build(addr, 20, vals, voff, N, hash_keys=True)
    root = hh[0].tobytes()
    assert st.n_leaves == N
    pinned = bytes.fromhex(PINNED_ROOTS[(CFG, N)])
    assert root == pinned, root.hex()
    a = addr[:20 * N].cpu().numpy()
    vo = voff[:N + 1].cpu().numpy().astype(np.uint64)
    vb = vals[:int(vo[N])].cpu().numpy()
    del addr, vals, voff
    ctx.close()
    torch.cuda.empty_cache()
    t0 = time.perf_counter()
    cpu, cst = oracle.batch_roots(a, (vb, vo), klen=20, hash_keys=True, nthreads=16)
    print(f"cpu batch builder: {time.perf_counter() - t0:.1f} s", flush=True)
    assert cpu[0] == root
    assert cst["distinct"] == N and cst["node_hashes"] == st.n_node_hashes
    # eight owner shards on one GPU: slices of 12.5M puts staged from host memory, hashed,
    # partitioned by owner (q * 8 >> 4), exchanged by device copies, built from depth 1
    s8 = KhStats()
    t0 = time.perf_counter()
    assert trie_root_sharded(a, (vb, vo), [0] * 8, hash_keys=True, klen=20, stats=s8) == root
    print(f"kh_trie_root_sharded x8: {time.perf_counter() - t0:.1f} s", flush=True)
    assert s8.n_inputs == N and s8.n_leaves == N


@pytest.mark.timeout(900)
def test_config4_torch_world8_at_size():
    """bench.py --gpus 8's driver at 100M: 8 rank processes of 12.5M accounts each on the one
    GPU, collectives host-staged over gloo; every rank's root == the pinned root, rank 0's
    single-GPU rebuild of all 100M accounts too."""
    import torch.multiprocessing as mp
    from khipu_amd.sharded import PINNED_ROOTS
    from tests.test_gpu_sharded_torch import _free_port, _worker
    world = 8
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, N, 0, q, False)) for r in range(world)]
    for p in procs:
        p.start()
    try:
        outs = [q.get(timeout=600) for _ in procs]
    finally:
        for p in procs:
            p.join(60)
            if p.exitcode is None:
                p.kill()
    errs = [o for o in outs if "error" in o]
    assert not errs, errs
    pinned = PINNED_ROOTS[(CFG, N)]
    assert {r for o in outs for r in o["roots"]} == {pinned}
    r0 = next(o for o in outs if o["rank"] == 0)
    assert r0["self_check"] and r0["single"] == pinned
    assert sum(o["leaves"] for o in outs) == N
