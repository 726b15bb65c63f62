"""One rank's share of the N-GPU sharded step, on one GPU (the exchange excluded):

  hash      kec256 of the rank's 100M/N slice of the addresses;
  partition the slice into N owners (kh_dev_partition_ev: keys, lengths, counts; the value
            copy, which the step overlaps with the key exchange, is timed on its own); and
            both in one call (kh_dev_hash_partition_ev: the hashing pass writes each key's
            owner byte for the count pass -- what the step runs since round 4);
  build     the OWNER-SHAPED shard from nibble 1 (depth0 = 1): the records of all 100M
            accounts whose top key nibble q has q * N >> 4 == 0 -- exactly what rank 0
            receives (100M/N records under 16/N root nibbles), not the rank's own slice.

Per-phase times are HIP-synchronised wall clock, median of the steps; the build's own
stage times come from its HIP events.  The exchange needs N GPUs: its bytes per peer are
reported and DESIGN.md §6 prices them from the xGMI link rate.  Prints one JSON line.

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
    p.add_argument("--cfg", type=int, default=5)
    a = p.parse_args()
    import numpy as np
    import torch
    from khipu_amd import sharded
    be = sharded.GpuBackend(0)
    N = a.world
    n = a.accounts // N
    # the owner-shaped shard: every account of the workload routed to owner 0 (source-major,
    # as the exchange delivers them), built once from the full synthetic set
    A, V, O = be.ctx.synth_accounts(a.cfg, 0, a.accounts)
    K = be.hash_keys(A, a.accounts)
    be.overlap = False
    pk, pv, pl, cnt, nb = be.partition(K, V, O, a.accounts, N)
    m = int(cnt[0])
    sk = pk[:32 * m + 64].clone()
    sv = pv[:int(nb[0]) + 64].clone()
    so = torch.zeros(m + 1, dtype=torch.int64, device=be.device)
    torch.cumsum(pl[:m], 0, out=so[1:])
    del A, V, O, K, pk, pv, pl
    torch.cuda.empty_cache()
    # this rank's own slice for the source-side phases
    addr, vals, voff = be.ctx.synth_accounts(a.cfg, 0, n)
    be.sync()
    times = {"hash_keys": [], "partition_keys": [], "value_copy": [], "build": [], "hash_partition_keys": []}
    hh = None
    for _ in range(a.steps + 1):
        t0 = time.perf_counter()
        k = be.hash_keys(addr, n)
        be.sync()
        t1 = time.perf_counter()
        be.overlap = True  # returns once keys, lengths and counts are in place
        _, _, _, c2, b2 = be.partition(k, vals, voff, n, N)
        t2 = time.perf_counter()
        be.vals_done.synchronize()
        be.sync()
        t3 = time.perf_counter()
        hh, ll, ii = be.build(sk, sv, so, m, depth0=1)
        be.sync()
        t4 = time.perf_counter()
        be.hash_partition(addr, vals, voff, n, N)  # hashing + partition in one call (the step's form)
        t5 = time.perf_counter()
        be.vals_done.synchronize()
        be.sync()
        for name, x, y in (("hash_keys", t0, t1), ("partition_keys", t1, t2), ("value_copy", t2, t3),
                           ("build", t3, t4), ("hash_partition_keys", t4, t5)):
            times[name].append((y - x) * 1e3)
    st = be.last_stats
    med = {k: round(float(np.median(v[1:])), 3) for k, v in times.items()}
    key_bytes_peer = int(c2[1:].sum()) * 32 // max(N - 1, 1) if N > 1 else 0
    val_bytes_peer = (int(c2[1:].sum()) * 8 + int(b2[1:].sum())) // max(N - 1, 1) if N > 1 else 0
    out = {"world": N, "records_per_rank": n, "shard_records": m,
           "shard_nibbles": [q for q in range(16) if (q * N) >> 4 == 0],
           "ms": med,
           # the step's form (sharded.sharded_root: one hash + partition call), and the two calls
           "critical_path_ms_excl_exchange": round(med["hash_partition_keys"] + med["build"], 3),
           "critical_path_ms_excl_exchange_two_calls": round(med["hash_keys"] + med["partition_keys"] + med["build"],
                                                             3),
           "build_stages_ms": {"sort": st.t_sort_ms, "topology": st.t_topo_ms, "leaves": st.t_leaf_ms,
                               "branches": st.t_branch_ms, "total": st.t_total_ms},
           "subtrie_refs_occupied": int((ll > 0).sum()),
           "exchange_bytes_per_peer": {"keys": key_bytes_peer, "lengths_and_values": val_bytes_peer},
           "owner_counts_of_slice": [int(x) for x in c2]}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
