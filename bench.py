"""bench.py — state-root throughput of libkhst.so on MI355X.

Metric (BASELINE.json): node-hashes/sec + full state-root time, 100M-account
trie.  One step = one full state root from (address, account body) pairs already
resident in HBM: kec256 of every address, sort, topology, RLP encode and
Keccak-256 of every node, bottom-up, to the root (hash_keys=True, as
TrieAccounts.flush -> MerklePatriciaTrie.put does via Address.hashedAddressEncoder).

N = 1: the whole 100M-account trie on one GPU (fits in 288 GB).
N > 1: (torch.distributed.run, one rank per GPU, RCCL) the same 100M trie with
each rank holding 1/N of the accounts: keys are routed to their top-nibble
owner with one all-to-all, each rank builds its 16/N subtries, the 16
references are all-gathered and folded into the root (khipu_amd/sharded.py).
Total work is fixed as N grows: "scaling": "strong".

Prints ONE JSON line (rank 0).
"""
import argparse
import json
import os
import platform
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

# Roofline constants (MI355X_MICROARCH.md): 256 CUs x 4 SIMD-32 x 2.4 GHz; a wave64
# VALU op issues in 2 cycles per SIMD (the same rate that gives the 157.3 TFLOPS FP32
# vector peak = 78.6 T lane-FMA/s), so the int32 VALU peak is 78.6 T lane-ops/s.
VALU_PEAK_LANE_OPS = 256 * 4 * 32 * 2.4e9
HBM_PEAK = 8.0e12
OPS_PER_PERM = 5760  # 24 rounds x 240 int32 ops


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=5)
    p.add_argument("--warmup", type=int, default=2)
    p.add_argument("--accounts", type=int, default=100_000_000)
    p.add_argument("--cfg", type=int, default=5, help="synthetic config id (SURVEY §8d seed)")
    p.add_argument("--cpu-sample", type=int, default=150_000, help="accounts in the CPU-baseline sample")
    p.add_argument("--no-cpu", action="store_true")
    p.add_argument("--sharded", action="store_true", help="force the nibble-sharded RCCL path (any N)")
    return p.parse_args()


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor()


def cpu_baseline(ctx, cfg, n_sample):
    """khipu-faithful sequential trie (oracle, 1 core) on the first n_sample accounts of
    the same synthetic workload, key hashing included; unit: node-hashes/s."""
    from oracle import oracle
    addr, vals, voff = ctx.synth_accounts(cfg, 0, n_sample)
    a = addr[:20 * n_sample].cpu().numpy().reshape(n_sample, 20)
    vo = voff.cpu().numpy().astype(np.uint64)
    vb = vals[:int(vo[n_sample])].cpu().numpy()
    # the same sample on the GPU gives the algorithmic node-hash count
    _, _, _, st = ctx.build(addr, 20, vals, voff, n_sample, hash_keys=True)
    t0 = time.perf_counter()
    keys = np.frombuffer(b"".join(oracle.kec256(x.tobytes()) for x in a), np.uint8)
    root = oracle.seq_root_packed(keys, 32, vb, vo, n_sample)
    dt = time.perf_counter() - t0
    hh, _, _, _ = ctx.build(addr, 20, vals, voff, n_sample, hash_keys=True)
    assert hh[0].tobytes() == root, "GPU/CPU root mismatch on the baseline sample"
    return {"value": st.n_node_hashes / dt, "unit": "node-hashes/s", "cores": 1, "kind": "port",
            "sample": f"first {n_sample} accounts of the same synthetic workload, sequential put per account "
                      f"(MerklePatriciaTrie.scala:157-281 as driven by TrieAccounts.flush), key hashing included; "
                      f"{dt:.2f} s, {dt / n_sample * 1e6:.2f} us/account, CPU: {cpu_model()}",
            "seconds": dt, "state_root_s_extrapolated_100M": dt / n_sample * 1e8}


def pmc_traffic(kernel, n):
    """HBM bytes per launch of `kernel` from the newest committed PMC summary of this
    workload size (profiles/*_pmc_traffic_<n>.json, written by scripts/pmc_summary.py
    from scripts/gpu_pmc.sh: read = 2 x FETCH_SIZE, write = WRITE_SIZE per
    MI355X_MICROARCH.md), or None when no pass was collected for it."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", f"*_pmc_traffic_{n}.json")))  # tags sort by round: newest last
    for f in reversed(files):
        with open(f) as fh:
            row = json.load(fh)["kernels"].get(kernel)
        if row and row.get("calls_per_build"):
            return row["hbm_bytes"] / row["calls_per_build"]
    return None


def single(args):
    import torch
    from khipu_amd.device import Ctx
    ctx = Ctx(0)
    n = args.accounts
    addr, vals, voff = ctx.synth_accounts(args.cfg, 0, n)
    torch.cuda.synchronize()
    for _ in range(args.warmup):
        ctx.build(addr, 20, vals, voff, n, hash_keys=True)
    torch.cuda.synchronize()
    stats = []
    t0 = time.perf_counter()
    for _ in range(args.steps):
        hh, ll, ii, st = ctx.build(addr, 20, vals, voff, n, hash_keys=True)
        stats.append(st.as_dict())
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / args.steps
    root = hh[0].tobytes().hex()
    s = stats[-1]
    ms_dev = float(np.mean([x["t_total_ms"] for x in stats]))
    # stage times (HIP events on the stream each stage runs on; k_leaf_fused runs on
    # the library's second stream, overlapped with the topology stage)
    stages = {"k_hash_keys": "t_keys_ms", "k_leaf_fused": "t_leaf_ms", "branch_levels": "t_branch_ms",
              "sort": "t_sort_ms", "topology": "t_topo_ms"}
    avg = {k: float(np.mean([x[v] for x in stats])) for k, v in stages.items()}
    # dominant single kernel: the larger of the two one-launch hash kernels
    dom = max(("k_hash_keys", "k_leaf_fused"), key=avg.get)
    perms = {"k_hash_keys": s["n_key_perms"], "k_leaf_fused": s["n_leaves"]}[dom]
    achieved = perms * OPS_PER_PERM / (avg[dom] * 1e-3)
    roof = {"kernel": dom, "bound": "valu", "achieved": achieved / 1e12, "peak": VALU_PEAK_LANE_OPS / 1e12,
            "unit": "T int32-lane-ops/s", "frac": achieved / VALU_PEAK_LANE_OPS,
            "traffic": pmc_traffic(dom, n), "avg_ms": avg[dom], "perms_per_launch": perms}
    out = {
        "metric": "node-hashes/sec (full state root, 100M-account trie)",
        "value": s["n_node_hashes"] / dt,
        "unit": "node-hashes/s",
        "n_gpus": 1, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": dt * 1e3,
        "higher_is_better": True, "scaling": "strong", "vs_baseline": None,
        "dtype": "u64", "data": "synthetic (counter-based accounts, SURVEY §8d, csrc/synth.h)",
        "config": {"workload": f"{n} synthetic accounts -> state root (keys hashed on GPU)", "accounts": n,
                   "parallelism": "single GPU"},
        "state_root": root,
        "device_ms_per_step": ms_dev,
        "stage_ms": avg,
        "topology": {k: s[k] for k in ("n_leaves", "n_branches", "n_extensions", "n_inline", "n_node_hashes",
                                       "n_node_perms", "n_key_perms", "arena_bytes", "n_levels")},
        "roofline": roof,
    }
    if not args.no_cpu:
        out["cpu_baseline"] = cpu_baseline(ctx, args.cfg, args.cpu_sample)
    print(json.dumps(out), flush=True)


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world > 1 or args.gpus > 1 or args.sharded:
        from khipu_amd import sharded
        sharded.bench_main(args)
    else:
        single(args)


if __name__ == "__main__":
    main()
