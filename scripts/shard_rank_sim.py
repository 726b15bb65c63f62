"""One rank's share of the N-GPU sharded step, on one GPU (the exchange excluded):
hash its 100M/N slice of the keys, partition the slice into N owners (kh_dev_partition),
then build a 100M/N-record shard from nibble 1 (depth0 = 1).  Prints per-phase times
(HIP-synchronised wall clock, median of the steps) as one JSON line.  The exchange
itself needs N GPUs; DESIGN.md §6 prices it from the xGMI link rate.

  python scripts/shard_rank_sim.py --world 8 [--accounts 100000000] [--steps 5]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--world", type=int, default=8)
    p.add_argument("--accounts", type=int, default=100_000_000)
    p.add_argument("--steps", type=int, default=5)
    p.add_argument("--cfg", type=int, default=1)
    a = p.parse_args()
    import numpy as np
    import torch
    from khipu_amd import sharded
    be = sharded.GpuBackend(0)
    n = a.accounts // a.world
    addr, vals, voff = be.ctx.synth_accounts(a.cfg, 0, n)
    be.sync()
    times = {"hash_keys": [], "partition": [], "build": []}
    for _ in range(a.steps + 1):
        t0 = time.perf_counter()
        k = be.hash_keys(addr, n)
        be.sync()
        t1 = time.perf_counter()
        pk, pv, pl, cnt, nb = be.partition(k, vals, voff, n, a.world)
        be.sync()
        t2 = time.perf_counter()
        # a shard of n records (this rank's slice stands in for what it would receive)
        vo = torch.zeros(n + 1, dtype=torch.int64, device=be.device)
        torch.cumsum(pl[:n], 0, out=vo[1:])
        be.sync()
        t3 = time.perf_counter()
        be.build(pk, pv, vo, n, depth0=1)
        be.sync()
        t4 = time.perf_counter()
        for name, x, y in (("hash_keys", t0, t1), ("partition", t1, t2), ("build", t3, t4)):
            times[name].append((y - x) * 1e3)
    st = be.last_stats
    out = {"world": a.world, "records_per_rank": n,
           "ms": {k: round(float(np.median(v[1:])), 3) for k, v in times.items()},
           "build_stages_ms": {"sort": st.t_sort_ms, "topology": st.t_topo_ms, "leaves": st.t_leaf_ms,
                               "branches": st.t_branch_ms, "total": st.t_total_ms},
           "value_bytes": int(nb.sum()), "owner_counts": [int(x) for x in cnt]}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
