"""One sample of the sequential CPU baseline (the khipu-faithful oracle, one core) beyond the
default bench samples: the first N accounts of the bench workload (csrc/synth.h config 5), keys
hashed inside the oracle's put loop (or_seq_root mode 2, as bench.py's cpu_baseline), its root
asserted equal to the GPU root of the same prefix.  Writes one JSON object; bench.py folds the
newest committed profiles/*_seq_sample_*.json into its fit of the per-put cost.
Measurement only (test infrastructure: the oracle is the thing timed, never shipped).

  python scripts/seq_sample.py --accounts 10000000 > profiles/r5x_seq_sample_10m.json

Prints a progress line to stderr every 60 s while the oracle runs (one C call)."""
import argparse
import json
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--accounts", type=int, default=10_000_000)
    p.add_argument("--cfg", type=int, default=5)
    a = p.parse_args()
    import numpy as np
    from bench import cpu_model, host_inputs
    from khipu_amd.device import Ctx
    from oracle import oracle
    n = a.accounts
    ctx = Ctx(0)
    addr, vals, voff = ctx.synth_accounts(a.cfg, 0, n)
    hh, _, _, st = ctx.build(addr, 20, vals, voff, n, hash_keys=True)
    gpu_root = hh[0].tobytes()
    k, vb, vo = host_inputs(addr, vals, voff, n)
    del addr, vals, voff
    out = {}

    def run():
        t0 = time.perf_counter()
        out["root"] = oracle.seq_root_packed(k, 20, vb, vo, n, mode=2)
        out["seconds"] = time.perf_counter() - t0

    th = threading.Thread(target=run)
    t0 = time.perf_counter()
    th.start()
    while th.is_alive():
        th.join(60)
        if th.is_alive():
            print(f"seq_sample: {n} accounts, {time.perf_counter() - t0:.0f} s", file=sys.stderr, flush=True)
    assert out["root"] == gpu_root, "GPU/CPU root mismatch"
    res = {"accounts": n, "seconds": round(out["seconds"], 3), "us_per_put": round(out["seconds"] / n * 1e6, 3),
           "node_hashes": int(st.n_node_hashes), "state_root": gpu_root.hex(), "state_root_match": True,
           "kind": "port", "cores": 1,
           "sample": f"first {n} accounts of bench.py's workload (config {a.cfg}), sequential put per account "
                     f"(MerklePatriciaTrie.scala:157-281 as driven by TrieAccounts.flush), key hashing included; "
                     f"CPU: {cpu_model()}"}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
