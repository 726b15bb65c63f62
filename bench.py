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
Total work is fixed as N grows: "scaling": "strong".  `python bench.py --gpus N`
without a launcher re-launches itself under torch.distributed.run (before any GPU
call) and exits with its status.

CPU legs (rank 0, N = 1, after the timed region):
  cpu_baseline       the khipu-faithful sequential trie (oracle/khipu_oracle.cc, 1 core)
                     on the first 20k/50k/100k/1M accounts of the same workload (--seq-samples);
                     every sample's root is asserted equal to the GPU root of the same prefix;
                     the 100M state-root time is extrapolated from the fitted per-put cost
  cpu_batch_allcore  the independent batch builder (oracle/batch_root.cc) on ALL cores
                     over the full workload; its root is asserted equal to the GPU root

Prints ONE JSON line (rank 0).
"""
import argparse
import json
import math
import os
import platform
import re
import socket
import subprocess
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
# The issue-rate floor of the permutation as this tree compiles it (keccak.h: 120 v_bitop3_b32,
# 58 v_alignbit_b32 and 2 v_xor a round) at the measured cycles per wave-instruction per SIMD
# with 8 waves per SIMD (profiles/r3zh_valu_issue_rates.txt: v_bitop3 2.61, v_alignbit 4.31 --
# the shifts issue at half rate -- v_xor 2.70), on the same 2.4 GHz basis as the peak
KECCAK_CYCLES_PER_WAVE_PERM = 24 * (120 * 2.61 + 58 * 4.31 + 2 * 2.70)


def issue_floor_ms(perms):
    """Time for `perms` permutations at the issue-rate floor (1,024 SIMDs at 2.4 GHz)."""
    return perms / 64 * KECCAK_CYCLES_PER_WAVE_PERM / (256 * 4 * 2.4e9) * 1e3
SEQ_SAMPLES = (20_000, 50_000, 100_000, 1_000_000)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=5)
    p.add_argument("--warmup", type=int, default=2)
    p.add_argument("--accounts", type=int, default=100_000_000)
    p.add_argument("--cfg", type=int, default=5, help="synthetic config id (SURVEY §8d seed)")
    p.add_argument("--seq-samples", type=str, default=",".join(map(str, SEQ_SAMPLES)),
                   help="account counts timed on the sequential CPU trie (comma separated)")
    p.add_argument("--cpu-threads", type=int, default=0, help="threads of the CPU batch builder (0: the box's share)")
    p.add_argument("--no-cpu", action="store_true")
    p.add_argument("--no-cpu-batch", action="store_true", help="skip the all-core full-size CPU root")
    p.add_argument("--sharded", action="store_true", help="force the nibble-sharded RCCL path (any N)")
    p.add_argument("--workload", choices=("state", "lists", "storage", "verify"), default="state",
                   help="state: the BASELINE metric (default); lists: transactions roots (SURVEY §8 f4); "
                        "storage: configs[3], 100k storage tries (trie-id shards over --gpus N); "
                        "verify: fast-sync NodeData verification (SURVEY §8 f3)")
    p.add_argument("--nodes-accounts", type=int, default=1_000_000,
                   help="verify: the NodeData batch is every node of a trie of this many accounts")
    p.add_argument("--no-host-path", action="store_true", help="state: skip the host-buffer (PCIe) drop-in timing")
    p.add_argument("--tries", type=int, default=100_000, help="storage: storage tries per step")
    p.add_argument("--blocks", type=int, default=10_000, help="lists: blocks per step")
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


def cpu_threads(req=0):
    """The box's CPU share: OMP_NUM_THREADS (16 per GPU on the pool), capped by affinity."""
    if req:
        return req
    try:
        avail = len(os.sched_getaffinity(0))
    except AttributeError:
        avail = os.cpu_count() or 1
    return max(1, min(avail, int(os.environ.get("OMP_NUM_THREADS", "16"))))


def fit_put_cost(samples):
    """Least-squares fit of us/put = a + b * log16(n) over (n, seconds) samples (the
    sequential put descends ~log16(n) levels).  Returns (a, b, residuals in us/put)."""
    xs = np.array([math.log(n, 16) for n, _ in samples])
    ys = np.array([t / n * 1e6 for n, t in samples])
    if len(samples) < 2:
        return float(ys[0]), 0.0, [0.0]
    A = np.stack([np.ones_like(xs), xs], 1)
    (a, b), *_ = np.linalg.lstsq(A, ys, rcond=None)
    res = ys - (a + b * xs)
    return float(a), float(b), [round(float(r), 4) for r in res]


def host_inputs(addr, vals, voff, n):
    a = addr[:20 * n].cpu().numpy()
    vo = voff[:n + 1].cpu().numpy().astype(np.uint64)
    vb = vals[:int(vo[n])].cpu().numpy()
    return a, vb, vo


def committed_seq_samples(cfg):
    """Samples of the same sequential port beyond the default ones (scripts/seq_sample.py,
    e.g. 10M accounts, ~10 minutes on one core): the newest committed
    profiles/*_seq_sample_*.json per size, each root asserted against the GPU when it was taken."""
    import glob
    out = {}
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_seq_sample_*.json")), key=round_key):
        try:
            with open(f) as fh:
                row = json.loads(fh.read().strip().splitlines()[-1])
        except (OSError, ValueError, IndexError):
            continue
        if row.get("state_root_match") and f"(config {cfg})" in row.get("sample", ""):
            out[row["accounts"]] = dict(row, source=os.path.relpath(f, ROOT))
    return [out[k] for k in sorted(out)]


def cpu_baseline(ctx, cfg, addr, vals, voff, samples):
    """khipu-faithful sequential trie (oracle, 1 core) on prefixes of the same synthetic
    workload, key hashing included; unit: node-hashes/s.  Asserts GPU == CPU per sample.
    The per-put cost fit also takes the committed larger samples (committed_seq_samples)."""
    from oracle import oracle
    rows = []
    for s in samples:
        _, _, _, st = ctx.build(addr, 20, vals, voff, s, hash_keys=True)  # algorithmic node-hash count
        hh, _, _, _ = ctx.build(addr, 20, vals, voff, s, hash_keys=True)
        a, vb, vo = host_inputs(addr, vals, voff, s)
        t0 = time.perf_counter()
        root = oracle.seq_root_packed(a, 20, vb, vo, s, mode=2)  # keys hashed in C, inside the put loop
        dt = time.perf_counter() - t0
        assert hh[0].tobytes() == root, f"GPU/CPU root mismatch on the {s}-account sample"
        rows.append({"accounts": s, "seconds": round(dt, 3), "us_per_put": round(dt / s * 1e6, 3),
                     "node_hashes": int(st.n_node_hashes)})
    a, b, res = fit_put_cost([(r["accounts"], r["seconds"]) for r in rows])
    big = rows[-1]
    est = 1e8 * (a + b * math.log(1e8, 16)) * 1e-6
    out = {"value": big["node_hashes"] / big["seconds"], "unit": "node-hashes/s", "cores": 1, "kind": "port",
           "sample": f"first {big['accounts']} accounts of the same synthetic workload, sequential put per account "
                     f"(MerklePatriciaTrie.scala:157-281 as driven by TrieAccounts.flush), key hashing included; "
                     f"{big['seconds']:.2f} s; GPU root asserted equal on every sample; CPU: {cpu_model()}",
           "samples": rows, "fit_us_per_put": {"a": round(a, 4), "b_per_log16n": round(b, 4),
                                               "residual_us_per_put": res},
           "state_root_s_extrapolated_100M": round(est, 1),
           "extrapolation": "100M x (a + b log16 100M) us from the fitted samples (not run)"}
    extra = [r for r in committed_seq_samples(cfg) if r["accounts"] > big["accounts"]]
    if extra:  # the slope pinned by the larger committed samples (timed on an earlier box)
        pts = [(r["accounts"], r["seconds"]) for r in rows] + [(r["accounts"], r["seconds"]) for r in extra]
        a2, b2, res2 = fit_put_cost(pts)
        est2 = 1e8 * (a2 + b2 * math.log(1e8, 16)) * 1e-6
        out["with_committed_samples"] = {
            "samples": [{k: r[k] for k in ("accounts", "seconds", "us_per_put", "source")} for r in extra],
            "fit_us_per_put": {"a": round(a2, 4), "b_per_log16n": round(b2, 4), "residual_us_per_put": res2},
            "state_root_s_extrapolated_100M": round(est2, 1),
            "note": "the same fit with the larger committed samples (derived: their times come from the box that "
                    "took them, named in source; this run's own samples are the ones above)"}
    return out


def host_path(addr, vals, voff, n, gpu_root, reps=2):
    """The JNI drop-in path: kh_trie_root from HOST buffers -- the addresses,
    the packed account bodies and their offsets staged over PCIe by the library, keys hashed on
    the GPU, the root back -- timed end to end on the wall clock (never `value`)."""
    from khipu_amd import trie as ktrie
    a, vb, vo = host_inputs(addr, vals, voff, n)
    times = []
    for _ in range(reps + 1):  # the first call also sizes the shared context's buffers
        t0 = time.perf_counter()
        root = ktrie.trie_root(a, (vb, vo), hash_keys=True, klen=20)
        times.append(time.perf_counter() - t0)
    assert root == gpu_root, "host-buffer root differs from the device-buffer root"
    h2d = a.nbytes + vb.nbytes + vo.nbytes
    best = min(times[1:])
    return {"ms": round(best * 1e3, 2), "ms_all": [round(t * 1e3, 2) for t in times], "h2d_bytes": int(h2d),
            "h2d_gb_per_s_if_all_copy": round(h2d / best / 1e9, 2), "state_root_match": True,
            "note": "kh_trie_root over pageable host arrays (the JVM's direct buffers): the library streams them "
                    "through pinned 64-MB chunks behind the build (keys in parts as hashing starts, then offsets, "
                    "values last, the leaves launched when they land); PCIe staging + the build on the wall clock; "
                    "not the bench value, whose inputs are already in HBM"}


def verify(args):
    """f3: fast-sync NodeData verification (kh_verify_nodes; NodeDatasRequest.processResponse,
    sync/package.scala:81-165) of one peer batch: every node of a synthetic state trie of
    --nodes-accounts accounts (kh_trie_root_nodes), requested as StateMptNodeHash, answered in
    a shuffled order.  One step = one kh_verify_nodes call from host buffers (PCIe staging
    included).  CPU leg: the oracle's restatement (or_verify_nodes) on one core over the same
    batch; every output is asserted equal."""
    import ctypes
    import torch
    from khipu_amd.device import Ctx
    from khipu_amd.trie import trie_root_nodes
    from khipu_amd._lib import check, lib
    ctx = Ctx(0)
    na = args.nodes_accounts
    addr, vals, voff = ctx.synth_accounts(args.cfg, 0, na)
    a, vb, vo = host_inputs(addr, vals, voff, na)
    _, nodes = trie_root_nodes([a[20 * i:20 * i + 20].tobytes() for i in range(na)],
                               [vb[vo[i]:vo[i + 1]].tobytes() for i in range(na)], hash_keys=True)
    rng = np.random.default_rng(7)
    hashes = list(nodes.keys())
    order = rng.permutation(len(hashes))
    values = [nodes[hashes[i]] for i in order]
    n = len(values)
    data = np.frombuffer(b"".join(values) + bytes(16), np.uint8)
    off = np.concatenate([[0], np.cumsum([len(v) for v in values])]).astype(np.uint64)
    req = np.frombuffer(b"".join(hashes), np.uint8)
    kinds = np.zeros(n, np.uint8)  # StateMptNodeHash
    hh = np.zeros((n, 32), np.uint8)
    match = np.zeros(n, np.int64)
    status = np.zeros(n, np.uint8)
    coff = np.zeros(n + 1, np.uint64)
    cap = 16 * n
    child = np.zeros((cap, 32), np.uint8)
    ckind = np.zeros(cap, np.uint8)
    total = ctypes.c_uint64()

    def call():  # kh_verify_nodes_packed: the children concatenated as processResponse lists them
        check(lib().kh_verify_nodes_packed(data.ctypes.data, off.ctypes.data, n, req.ctypes.data, kinds.ctypes.data,
                                           n, hh.ctypes.data, match.ctypes.data, status.ctypes.data,
                                           coff.ctypes.data, child.ctypes.data, ckind.ctypes.data, cap,
                                           ctypes.byref(total)))
    for _ in range(args.warmup):
        call()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        call()
    dt = (time.perf_counter() - t0) / args.steps
    out = {"metric": "fast-sync NodeData values verified/s (kec256 + request match + PV63 decode)", "value": n / dt,
           "unit": "nodes/s", "n_gpus": 1, "steps": args.steps, "warmup": args.warmup, "ms_per_step": dt * 1e3,
           "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u64",
           "data": "synthetic (every node of a state trie of synthetic accounts, shuffled)",
           "config": {"workload": f"{n} NodeData values ({int(off[-1])} B) of a {na}-account state trie, one "
                                  f"kh_verify_nodes call from host buffers", "nodes": n, "bytes": int(off[-1]),
                      "parallelism": "single GPU"},
           "children_listed": int(total.value)}
    assert (match >= 0).all() and (status == 0).all()
    nchild = np.diff(coff).astype(np.uint8)
    if not args.no_cpu:
        from oracle import oracle
        t1 = time.perf_counter()
        ch, cm, cs, cn, cc, ck = oracle.verify_nodes_batch(data, off, req, kinds)
        tc = time.perf_counter() - t1
        assert (ch == hh).all() and (cm == match).all() and (cs == status).all() and (cn == nchild).all()
        mask = np.arange(16)[None, :] < nchild[:, None]
        t = int(total.value)
        assert (cc[mask] == child[:t]).all() and (ck[mask] == ckind[:t]).all()  # row-major = concatenation order
        out["cpu_baseline"] = {"value": n / tc, "unit": "nodes/s", "cores": 1, "kind": "port",
                               "sample": f"the same {n} values, or_verify_nodes (NodeDatasRequest.processResponse "
                                         f"restated, one core); every output asserted equal; CPU: {cpu_model()}",
                               "seconds": round(tc, 3)}
    print(json.dumps(out), flush=True)


def cpu_batch(addr, vals, voff, n, gpu_root, threads):
    """Independent batch builder (oracle/batch_root.cc) on all of the box's cores over the
    full workload; asserts its root equals the GPU's."""
    from oracle import oracle
    a, vb, vo = host_inputs(addr, vals, voff, n)
    t0 = time.perf_counter()
    roots, st = oracle.batch_roots(a, (vb, vo), klen=20, hash_keys=True, nthreads=threads)
    dt = time.perf_counter() - t0
    ok = roots[0] == gpu_root
    del a, vb, vo
    assert ok, f"GPU root {gpu_root.hex()} != CPU batch root {roots[0].hex()} at {n} accounts"
    return {"value": st["node_hashes"] / dt, "unit": "node-hashes/s", "cores": threads, "kind": "port",
            "seconds": round(dt, 3), "state_root_match": True, "node_hashes": st["node_hashes"],
            "node_perms": st["node_perms"], "key_perms": st["key_perms"],
            "sample": f"all {n} accounts (the full workload), sort + bottom-up hash on {threads} threads, "
                      f"key hashing included; CPU: {cpu_model()}"}


def round_key(path):
    """profiles/r<round><letters>_... -> (round, letters): r10a sorts after r2b."""
    m = re.match(r"r(\d+)([a-z]*)_", os.path.basename(path))
    return (int(m.group(1)), m.group(2)) if m else (-1, "")


def pmc_traffic(kernel, n):
    """HBM bytes per launch of `kernel` from the newest committed PMC summary of this
    workload size (profiles/*_pmc_traffic_<n>.json, written by scripts/pmc_summary.py
    from scripts/gpu_pmc.sh: read = 2 x FETCH_SIZE, write = WRITE_SIZE per
    MI355X_MICROARCH.md), or None when no pass was collected for it."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", f"*_pmc_traffic_{n}.json")), key=round_key)
    for f in reversed(files):
        with open(f) as fh:
            row = json.load(fh)["kernels"].get(kernel)
        if row and row.get("calls_per_build"):
            return row["hbm_bytes"] / row["calls_per_build"]
    return None


def pmc_traffic_per_unit(kernel, units_per_launch):
    """HBM bytes per launch of `kernel` for a launch of `units_per_launch` units, scaled from the
    newest committed 100M PMC summary (the leaf kernel's bytes per leaf do not depend on the
    size: input-order reads, one scattered 32-byte stash per leaf).  The sharded lines use it
    for their per-rank launches; None without a summary."""
    full = pmc_traffic(kernel, 100_000_000)
    if full is None:
        return None
    return full / 100_000_000 * units_per_launch


def committed_cpu_baseline():
    """The cpu_baseline of the newest committed N = 1 bench line (profiles/r*_bench*.json):
    the sequential port is timed on rank 0 at N = 1 only (its 4-sample fit up to 1M accounts);
    the N > 1 lines report that measurement, named by its file, instead of timing it again."""
    import glob
    best = None
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_bench*.json")), key=round_key):
        try:
            with open(f) as fh:
                row = json.loads(fh.read().strip().splitlines()[-1])
        except (OSError, ValueError, IndexError):
            continue
        cb = row.get("cpu_baseline")
        if row.get("n_gpus") == 1 and cb and row.get("metric", "").startswith("node-hashes/sec (full state root"):
            best = dict(cb, source=f"{os.path.relpath(f, ROOT)} (timed at N = 1 on rank 0; not re-run at N > 1)")
    return best


def roofline(stats, n):
    """Dominant single kernel of the step (the larger of the two one-launch hash kernels),
    from the HIP events the library records on the stream each kernel runs on."""
    stages = {"k_hash_keys_ck": "t_keys_ms", "k_leaf_in": "t_leaf_ms", "branch_levels": "t_branch_ms",
              "sort": "t_sort_ms", "topology": "t_topo_ms"}
    avg = {k: float(np.mean([x[v] for x in stats])) for k, v in stages.items()}
    s = stats[-1]
    total = {"k_hash_keys_ck": avg["k_hash_keys_ck"], "k_leaf_in": avg["k_leaf_in"]}
    dom = max(total, key=total.get)
    perms = {"k_hash_keys_ck": s["n_key_perms"], "k_leaf_in": s["n_leaves"]}[dom]
    launch_ms = total[dom]
    achieved = perms * OPS_PER_PERM / (launch_ms * 1e-3)
    return avg, {"kernel": dom, "bound": "valu", "achieved": achieved / 1e12, "peak": VALU_PEAK_LANE_OPS / 1e12,
                 "unit": "T int32-lane-ops/s", "frac": achieved / VALU_PEAK_LANE_OPS,
                 "traffic": pmc_traffic(dom, n), "avg_ms": launch_ms, "launches_per_step": 1,
                 "perms_per_launch": perms,
                 "issue_floor": {"ms": issue_floor_ms(perms), "frac": issue_floor_ms(perms) / launch_ms,
                                 "basis": "the launch's permutations alone at the measured issue rates of the "
                                          "instructions the permutation compiles to (v_alignbit at half rate; "
                                          "bench.py KECCAK_CYCLES_PER_WAVE_PERM)"}}


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
    root = hh[0].tobytes()
    s = stats[-1]
    ms_dev = float(np.mean([x["t_total_ms"] for x in stats]))
    avg, roof = roofline(stats, n)
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
        "state_root": root.hex(),
        "device_ms_per_step": ms_dev,
        "stage_ms": avg,
        "topology": {k: s[k] for k in ("n_leaves", "n_branches", "n_extensions", "n_inline", "n_node_hashes",
                                       "n_node_perms", "n_key_perms", "arena_bytes", "n_levels")},
        "roofline": roof,
        # each Keccak stage against its permutations' issue-rate floor (the leaves' and the levels'
        # encoding work, loads and stores are on top of the floor: frac < 1 is that, plus stalls)
        "issue_floor_by_stage": {
            k: {"perms": p, "ms": avg[m], "floor_ms": issue_floor_ms(p), "frac": issue_floor_ms(p) / max(avg[m], 1e-9)}
            for k, m, p in (("key_hashing", "k_hash_keys_ck", s["n_key_perms"]), ("leaves", "k_leaf_in", s["n_leaves"]),
                            ("branch_levels", "branch_levels", s["n_node_perms"] - s["n_leaves"]))},
    }
    if not args.no_host_path:
        out["drop_in_host_path"] = host_path(addr, vals, voff, n, root)
    if not args.no_cpu:
        samples = [int(x) for x in args.seq_samples.split(",") if x and int(x) <= n]
        if samples:
            out["cpu_baseline"] = cpu_baseline(ctx, args.cfg, addr, vals, voff, samples)
        if not args.no_cpu_batch:
            out["cpu_batch_allcore"] = cpu_batch(addr, vals, voff, n, root, cpu_threads(args.cpu_threads))
            out["parity"] = {"full_size_root_vs_cpu_batch": "equal"}
    print(json.dumps(out), flush=True)


def list_workload(nblk, seed=11):
    """nblk blocks of 1..300 transactions (mean ~150) of 100..220 bytes each (signed
    transactions), packed: (items uint8, item offsets uint64[n+1], block offsets uint64[nblk+1])."""
    r = np.random.default_rng(seed)
    cnt = r.integers(1, 301, nblk)
    so = np.zeros(nblk + 1, np.uint64)
    so[1:] = np.cumsum(cnt)
    n = int(so[-1])
    ln = r.integers(100, 221, n)
    off = np.zeros(n + 1, np.uint64)
    off[1:] = np.cumsum(ln)
    items = r.integers(0, 256, int(off[-1]) + 64, dtype=np.uint8)
    return items, off, so


def lists(args):
    """f4: every block's transactions root (MptListValidator.scala:15-46) for `--blocks`
    blocks in one kh_dev_list_roots call (items already in HBM; rlp(i) keys made on the
    device).  CPU legs: the batch builder over the same lists on all cores, and the
    sequential khipu-faithful fold on a 200-block sample; every root is asserted equal."""
    import torch
    from khipu_amd.device import Ctx
    ctx = Ctx(0)
    items, off, so = list_workload(args.blocks)
    n, nblk = int(so[-1]), len(so) - 1
    d_items = torch.from_numpy(items).to("cuda:0")
    d_off = torch.from_numpy(off.astype(np.int64)).to("cuda:0")
    for _ in range(args.warmup):
        ctx.list_roots(d_items, d_off, so)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        roots, st = ctx.list_roots(d_items, d_off, so)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / args.steps
    s = st.as_dict()
    perms_leaf = s["n_leaves"]
    leaf_ms = s["t_leaf_ms"]
    achieved = perms_leaf * OPS_PER_PERM / max(leaf_ms * 1e-3, 1e-12)
    out = {
        "metric": "list-roots/sec (transactions roots, rlp(i) keys)", "value": nblk / dt, "unit": "roots/s",
        "n_gpus": 1, "steps": args.steps, "warmup": args.warmup, "ms_per_step": dt * 1e3, "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "u64",
        "data": "synthetic (1..300 transactions of 100..220 random bytes per block)",
        "config": {"workload": f"{nblk} blocks, {n} transactions -> one transactions root per block",
                   "blocks": nblk, "items": n, "parallelism": "single GPU"},
        "items_per_s": n / dt, "node_hashes": s["n_node_hashes"], "device_ms_per_step": s["t_total_ms"],
        "stage_ms": {k: s[k] for k in ("t_keys_ms", "t_sort_ms", "t_topo_ms", "t_leaf_ms", "t_branch_ms")},
        "roofline": {"kernel": "k_leaf_prep+k_leaf_hash", "bound": "valu", "achieved": achieved / 1e12,
                     "peak": VALU_PEAK_LANE_OPS / 1e12, "unit": "T int32-lane-ops/s",
                     "frac": achieved / VALU_PEAK_LANE_OPS, "traffic": None,
                     "note": "leaf stage priced on one permutation per leaf (long leaves take two)"},
    }
    if not args.no_cpu:
        from oracle import oracle
        keys = []
        for b in range(nblk):
            keys += [oracle_list_key(i) for i in range(int(so[b + 1] - so[b]))]
        threads = args.cpu_threads or min(16, os.cpu_count() or 1)
        t1 = time.perf_counter()
        croots, _ = oracle.batch_roots(keys, (items, off), seg_off=so, nthreads=threads)
        tb = time.perf_counter() - t1
        assert croots == roots, "GPU list roots differ from the CPU batch builder"
        sample = min(200, nblk)
        t2 = time.perf_counter()
        for b in range(sample):
            t = oracle.Trie()
            for i in range(int(so[b + 1] - so[b])):
                j = int(so[b]) + i
                t.put(oracle_list_key(i), items[int(off[j]):int(off[j + 1])].tobytes())
            assert t.root_hash() == roots[b], f"block {b}: GPU root differs from the sequential fold"
        ts = time.perf_counter() - t2
        out["cpu_baseline"] = {"value": sample / ts, "unit": "roots/s", "cores": 1, "kind": "port",
                               "sample": f"the first {sample} blocks of the same lists, sequential put of every "
                                         f"item (MerklePatriciaTrie.put, MptListValidator.scala:30-46); "
                                         f"{ts:.2f} s; every root asserted equal; CPU: {cpu_model()}"}
        out["cpu_batch_allcore"] = {"value": nblk / tb, "unit": "roots/s", "cores": threads, "kind": "port",
                                    "seconds": round(tb, 3), "roots_match": True,
                                    "sample": "all blocks, independent batch builder (oracle/batch_root.cc)"}
    print(json.dumps(out), flush=True)


def storage_ranges(seg_off, world):
    """Contiguous trie ranges [b[g], b[g+1]) of about equal slot counts (seg_off: the tries'
    slot offsets, nt + 1 entries from 0), one per rank; every trie in exactly one range."""
    nt = len(seg_off) - 1
    tot = int(seg_off[-1])
    b = [0] + [int(np.searchsorted(seg_off, tot * g // world, side="left")) for g in range(1, world)] + [nt]
    for g in range(1, world + 1):
        b[g] = min(max(b[g], b[g - 1]), nt)
    return b


def storage(args):
    """configs[3]: the roots of 100k synthetic contract storage tries (csrc/synth.h: log-uniform
    1..10^4 slots, kec256 slot keys hashed on the GPU, RLP(trimmed 1-32 B) values) as one
    segmented build per GPU.  N > 1 (torch.distributed, one rank per GPU): the tries are split
    into contiguous ranges of equal slot counts, each rank generates and builds its own range,
    and the roots are gathered (SURVEY §8e "Other configs": no exchange, the tries are
    independent; TrieStorage.scala:52-60 via BlockWorldState.scala:243-252).  Total work is
    fixed as N grows ("strong").  Rank 0 checks the gathered roots against a single-GPU build
    of all tries and, at N = 1, against the CPU batch builder."""
    import torch
    import torch.distributed as dist
    from khipu_amd.device import Ctx
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device(f"cuda:{local}"))
    ctx = Ctx(local)
    cfg, NT = 4, args.tries
    so_all, n_all, _ = ctx.storage_slot_counts(cfg, 0, NT)
    so_h = so_all.cpu().numpy()
    bnd = storage_ranges(so_h, world)
    t0, t1 = bnd[rank], bnd[rank + 1]
    nt = t1 - t0
    so, keys, vals, voff, seg = ctx.synth_storage(cfg, t0, nt)
    n = int(so[-1].item()) if nt else 0
    torch.cuda.synchronize()

    def step():
        return ctx.build(keys, 32, vals, voff, n, seg=seg, nseg=max(nt, 1), hash_keys=True) if n else None

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t_0 = time.perf_counter()
    dev_ms = []
    for _ in range(args.steps):
        out = step()
        if out:
            dev_ms.append(out[3].t_total_ms)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t_0) / args.steps
    hh = out[0][:nt] if out else np.zeros((0, 32), np.uint8)
    st = out[3].as_dict() if out else None
    mine = np.zeros((max(bnd[g + 1] - bnd[g] for g in range(world)), 32), np.uint8)
    mine[:nt] = hh
    hashes = st["n_node_hashes"] if st else 0
    if world > 1:
        dtt = torch.tensor([dt], dtype=torch.float64, device=f"cuda:{local}")
        dist.all_reduce(dtt, op=dist.ReduceOp.MAX)
        dt = float(dtt.item())
        ht = torch.tensor([hashes], dtype=torch.int64, device=f"cuda:{local}")
        dist.all_reduce(ht)
        hashes = int(ht.item())
        allr = [torch.zeros_like(torch.from_numpy(mine)).to(f"cuda:{local}") for _ in range(world)]
        dist.all_gather(allr, torch.from_numpy(mine).to(f"cuda:{local}"))
        roots = np.concatenate([allr[g].cpu().numpy()[:bnd[g + 1] - bnd[g]] for g in range(world)])
    else:
        roots = hh
    ok = torch.ones(1, dtype=torch.int64, device=f"cuda:{local}")
    res = None
    if rank == 0:
        # self-check: every root against one single-GPU segmented build of ALL the tries
        if world > 1:
            del keys, vals, voff, seg
            torch.cuda.empty_cache()
        so1, k1, v1, o1, s1 = ctx.synth_storage(cfg, 0, NT)
        h1, _, _, st1 = ctx.build(k1, 32, v1, o1, n_all, seg=s1, nseg=NT, hash_keys=True)
        single_ok = bool((h1[:NT] == roots).all())
        ok[0] = int(single_ok)
        s = st1.as_dict()
        leaf_ms = s["t_leaf_ms"]
        achieved = s["n_leaves"] * OPS_PER_PERM / max(leaf_ms * 1e-3, 1e-12)
        res = {
            "metric": "node-hashes/sec (configs[3]: 100k storage tries, one root each)",
            "value": hashes / dt, "unit": "node-hashes/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": dt * 1e3, "higher_is_better": True, "scaling": "strong",
            "vs_baseline": None, "dtype": "u64",
            "data": "synthetic (counter-based storage tries, csrc/synth.h synth_storage_*)",
            "config": {"workload": f"{NT} storage tries, {n_all} slots (log-uniform 1..1e4 per trie) -> one root each",
                       "tries": NT, "slots": n_all,
                       "parallelism": f"trie-id shards x{world} (slot-balanced ranges, roots gathered)"},
            "trie_ranges": [[bnd[g], bnd[g + 1]] for g in range(world)],
            "rank0_device_ms_per_step": [round(x, 3) for x in dev_ms],
            "parity": {"roots_vs_single_gpu_build": "equal" if single_ok else "DIFFER"},
            "stage_ms_single_gpu_build": {k: round(s[k], 3) for k in ("t_keys_ms", "t_sort_ms", "t_topo_ms",
                                                                        "t_leaf_ms", "t_branch_ms", "t_total_ms")},
            "roofline": {"kernel": "k_leaf_in (single-GPU build of all tries)", "bound": "valu",
                         "achieved": achieved / 1e12, "peak": VALU_PEAK_LANE_OPS / 1e12,
                         "unit": "T int32-lane-ops/s", "frac": achieved / VALU_PEAK_LANE_OPS, "traffic": None,
                         "avg_ms": leaf_ms, "perms_per_launch": s["n_leaves"]},
        }
        if world == 1 and not args.no_cpu and single_ok:
            from oracle import oracle
            thr = cpu_threads(args.cpu_threads)
            vo = o1.cpu().numpy().astype(np.uint64)
            tc = time.perf_counter()
            cr, cst = oracle.batch_roots(k1[:32 * n_all].cpu().numpy(), (v1[:int(vo[-1])].cpu().numpy(), vo), klen=32,
                                         seg_off=so1.cpu().numpy().astype(np.uint64), hash_keys=True, nthreads=thr)
            tcpu = time.perf_counter() - tc
            cpu_ok = cr == [bytes(x) for x in h1[:NT]]
            ok[0] = int(cpu_ok)
            res["parity"]["roots_vs_cpu_batch"] = "equal" if cpu_ok else "DIFFER"
            res["cpu_baseline"] = {"value": cst["node_hashes"] / tcpu, "unit": "node-hashes/s", "cores": thr,
                                   "kind": "port", "seconds": round(tcpu, 3),
                                   "sample": f"all {NT} tries, independent batch builder (oracle/batch_root.cc) on "
                                             f"{thr} threads, key hashing included; CPU: {cpu_model()}"}
    if world > 1:
        dist.broadcast(ok, 0)
    if not int(ok.item()):
        if rank == 0:
            print(f"storage roots FAILED their self-check: {res and res['parity']}", file=sys.stderr, flush=True)
        if world > 1:
            dist.destroy_process_group()
        sys.exit(1)
    if rank == 0:
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def oracle_list_key(i):
    """rlp.encode(i: Int) (RLP.scala integer encoding): 0 -> 0x80, 1..127 the byte, else 0x80+len, BE bytes."""
    if i == 0:
        return b"\x80"
    if i < 0x80:
        return bytes([i])
    b = i.to_bytes((i.bit_length() + 7) // 8, "big")
    return bytes([0x80 + len(b)]) + b


def relaunch(args):
    """`bench.py --gpus N` without a launcher: start torch.distributed.run as a child (no
    GPU call has been made in this process) and exit with its status."""
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(cmd, env=env)


def keep_stdout_for_json():
    """Native libraries print banners on fd 1 (RCCL's version block at communicator
    creation): point fd 1 at stderr and keep Python's sys.stdout on the original stream,
    so stdout carries only the JSON line."""
    sys.stdout.flush()
    saved = os.dup(1)
    os.dup2(2, 1)
    sys.stdout = os.fdopen(saved, "w", buffering=1)


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(relaunch(args))
    keep_stdout_for_json()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if args.workload == "lists":
        lists(args)
    elif args.workload == "storage":
        storage(args)
    elif args.workload == "verify":
        verify(args)
    elif world > 1 or args.gpus > 1 or args.sharded:
        from khipu_amd import sharded
        sharded.bench_main(args)
    else:
        single(args)


if __name__ == "__main__":
    main()
