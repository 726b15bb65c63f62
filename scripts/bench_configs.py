"""Secondary workloads of BASELINE.json `configs` on one MI355X (bench.py measures configs[4]).

  --cfg 2  configs[1]: 1M synthetic accounts, full build + root (keys hashed on the GPU).
  --cfg 3  configs[2]: block commits over a resident state: N_RES
           accounts (default 50M) plus 2,000 resident 1k-slot storage tries; per block 20k
           dirty accounts (90% updates, 5% inserts, 5% deletes) and 10 dirty slots per
           contract, storage roots injected into the accounts, one kh_block_commit
           (tests/blocks.py).
  --cfg 4  configs[3]: 100k storage tries, slot counts log-uniform in [1, 1e4], slot key =
           kec256(32-byte BE slot index) (KH_HASH_KEYS), value = RLP(trimmed 1-32 random
           bytes), one segmented build; 4 segments re-built alone must give the same roots.

Inputs are generated on the device before the timed region.  Prints one JSON line per
config.  Parity of these paths is tests/test_gpu_configs.py, test_gpu_resident.py and
test_gpu_parity.py; here every root is also cross-checked against a from-scratch device
build of the same final set and (unless --no-cpu) against the independent CPU batch builder
(oracle/batch_root.cc: the 50M final state root, all 2,000 storage roots, all 100k
segmented roots).
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from khipu_amd._lib import check, lib  # noqa: E402
from khipu_amd.device import Ctx, _ptr  # noqa: E402

DEV = "cuda:0"


def hash_keys(ctx, d_in, klen, n):
    out = torch.empty(n * 32 + 64, dtype=torch.uint8, device=DEV)
    torch.cuda.synchronize()
    check(lib().kh_dev_hash_keys(ctx.h, _ptr(d_in), klen, n, _ptr(out)))
    torch.cuda.synchronize()
    return out


def storage_values(g, n):
    """RLP(trimmed 1-32 random bytes) per slot (rlpDataWordSerializer, trie/package.scala:28-32):
    a single byte < 0x80 is its own encoding, otherwise 0x80+L then the L bytes."""
    L = torch.randint(1, 33, (n,), generator=g, device=DEV)
    b0 = torch.randint(1, 256, (n,), generator=g, device=DEV)
    raw = (L == 1) & (b0 < 0x80)
    elen = torch.where(raw, 1, L + 1)
    voff = torch.zeros(n + 1, dtype=torch.int64, device=DEV)
    voff[1:] = torch.cumsum(elen, 0)
    tot = int(voff[-1])
    vals = torch.randint(0, 256, (tot + 64,), generator=g, device=DEV, dtype=torch.uint8)
    st = voff[:-1]
    pre = ~raw
    vals[st[pre]] = (0x80 + L[pre]).to(torch.uint8)
    vals[st + pre.long()] = b0.to(torch.uint8)
    return vals, voff


def slot_keys(idx):
    """32-byte big-endian slot indices (DataWord, hashed by hashDataWordSerializable)."""
    n = idx.numel()
    k = torch.zeros(n, 32, dtype=torch.uint8, device=DEV)
    for b in range(8):
        k[:, 31 - b] = ((idx >> (8 * b)) & 0xFF).to(torch.uint8)
    return k.reshape(-1)


def seg_build(ctx, keys, vals, voff, seg, nseg, n):
    hh, ll, _, st = ctx.build(keys, 32, vals, voff, n, seg=seg, nseg=nseg, hash_keys=True)
    return hh, st


def cfg2(args):
    ctx = Ctx(0)
    n = 1_000_000
    addr, vals, voff = ctx.synth_accounts(2, 0, n)
    for _ in range(args.warmup):
        ctx.build(addr, 20, vals, voff, n, hash_keys=True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        hh, _, _, st = ctx.build(addr, 20, vals, voff, n, hash_keys=True)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / args.steps
    return {"config": "configs[1]: 1M synthetic accounts, full build + root", "ms": dt * 1e3,
            "device_ms": st.t_total_ms, "node_hashes": st.n_node_hashes, "node_hashes_per_s": st.n_node_hashes / dt,
            "state_root": hh[0].tobytes().hex()}


def cfg3(args):
    """configs[2] at its configured size: tests/blocks.py's workload over a 50M-account
    resident state trie with 2,000 resident 1k-slot storage tries; one kh_block_commit per
    block.  The final state root and every storage root are checked against from-scratch
    GPU builds of the final sets (parity of the same path at 1M against the CPU batch
    builder and the oracle: tests/test_gpu_configs.py::test_config2_block_commits)."""
    from tests.blocks import BlockWorkload
    ctx = Ctx(0)
    nb = args.warmup + args.steps
    t0 = time.perf_counter()
    w = BlockWorkload(ctx, args.resident, nb + 1, nc=args.contracts, dirty=args.dirty)
    open_s = time.perf_counter() - t0
    u_open = {"state": w.state.usage(), "storage": w.forest.usage()}
    for b in range(nb):
        root = w.block(b)
    blocks = w.t_commit[args.warmup:]
    ms = np.array([x[0] for x in blocks])
    # record / heap growth over the blocks, then one compaction of each handle (kh_trie_compact)
    # and one more block on the compacted records
    u_blocks = {"state": w.state.usage(), "storage": w.forest.usage()}
    torch.cuda.synchronize()
    tc0 = time.perf_counter()
    w.state.compact()
    tc1 = time.perf_counter()
    w.forest.compact()
    tc2 = time.perf_counter()
    u_compact = {"state": w.state.usage(), "storage": w.forest.usage()}
    root = w.block(nb)
    compaction = {
        "usage_after_open": u_open, "usage_after_blocks": u_blocks, "usage_after_compaction": u_compact,
        "dead_record_bytes_per_block": {k: (u_blocks[k]["records"] - u_blocks[k]["live_records"]
                                            - (u_open[k]["records"] - u_open[k]["live_records"])) * 128 // nb
                                        for k in u_open},
        "compact_ms": {"state": (tc1 - tc0) * 1e3, "storage": (tc2 - tc1) * 1e3},
        "block_ms_after_compaction": w.t_commit[-1][0],
    }
    K, V, O, N = w.final_accounts()
    hf, _, _, _ = ctx.build(K, 32, V, O, N)
    assert hf[0].tobytes() == root, "block-commit state root != full build of the final state"
    checked = f"state root and all {w.nc} storage roots == full GPU builds"
    if not args.no_cpu:  # the independent CPU batch builder over the whole final state
        from oracle import oracle
        vo = O.cpu().numpy().astype(np.uint64)
        tc = time.perf_counter()
        cpu, _ = oracle.batch_roots(K.cpu().numpy(), (V[:int(vo[-1])].cpu().numpy(), vo), klen=32,
                                    nthreads=args.cpu_threads)
        cpu_s = time.perf_counter() - tc
        assert cpu[0] == root, "block-commit state root != CPU batch build of the final state"
    del K, V, O
    K, V, O, T, N = w.final_storage()
    hh, _, _, _ = ctx.build(K, 32, V, O, N, seg=T, nseg=w.nc, hash_keys=True)
    bad = [c for c in range(w.nc) if hh[c].tobytes() != w.roots[c]]
    assert not bad, f"storage roots differ from full builds: {bad[:5]}"
    if not args.no_cpu:
        so = O.cpu().numpy().astype(np.uint64)
        seg_off = np.searchsorted(T.cpu().numpy(), np.arange(w.nc + 1)).astype(np.uint64)
        cs, _ = oracle.batch_roots(K.cpu().numpy(), (V[:int(so[-1])].cpu().numpy(), so), klen=32, seg_off=seg_off,
                                   hash_keys=True, nthreads=args.cpu_threads)
        bad = [c for c in range(w.nc) if cs[c] != w.roots[c]]
        assert not bad, f"storage roots differ from the CPU batch builder: {bad[:5]}"
        checked = (f"state root and all {w.nc} storage roots == full GPU builds AND == the CPU batch builder "
                   f"(oracle/batch_root.cc, {args.cpu_threads} threads, state root {cpu_s:.1f} s)")
    return {"config": f"configs[2]: {args.dirty} dirty accounts + {args.contracts} storage tries x 10 dirty slots per "
                      f"block over a {args.resident / 10**6:g}M-account resident trie (kh_block_commit)",
            "open_s": open_s, "block_ms_median": float(np.median(ms)), "block_ms_all": ms.tolist(),
            "rehashed_nodes_median": int(np.median([x[1] for x in blocks])),
            "ops_per_block": int(blocks[0][2]), "resident_accounts_after": len(w.state),
            "state_root_after": root.hex(), "checked": checked, "compaction": compaction}


def cfg4(args):
    ctx = Ctx(0)
    g = torch.Generator(device=DEV)
    g.manual_seed(4)
    nseg = 100_000
    u = torch.rand(nseg, generator=g, device=DEV, dtype=torch.float64)
    cnt = torch.clamp(torch.floor(torch.exp(u * np.log(1e4 + 1))), 1, 10_000).to(torch.int64)
    n = int(cnt.sum())
    seg = torch.arange(nseg, device=DEV, dtype=torch.int32).repeat_interleave(cnt)
    base = torch.zeros(nseg, dtype=torch.int64, device=DEV)
    base[1:] = torch.cumsum(cnt, 0)[:-1]
    idx = torch.arange(n, device=DEV, dtype=torch.int64) - base.repeat_interleave(cnt)
    keys = slot_keys(idx)
    del idx, base
    vals, voff = storage_values(g, n)
    for _ in range(args.warmup):
        seg_build(ctx, keys, vals, voff, seg, nseg, n)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        hh, st = seg_build(ctx, keys, vals, voff, seg, nseg, n)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / args.steps
    # four tries re-built alone (smallest, largest, two random) give the same roots
    c = cnt.cpu().numpy()
    offs = np.concatenate([[0], np.cumsum(c)])
    so = voff.cpu().numpy()
    checks = [int(np.argmin(c)), int(np.argmax(c)), 7, nseg - 3]
    kv = keys.view(n, 32)
    for s in checks:
        lo, hi = int(offs[s]), int(offs[s + 1])
        k1 = kv[lo:hi].reshape(-1).contiguous()
        v1 = vals[int(so[lo]):int(so[hi])].contiguous()
        o1 = (voff[lo:hi + 1] - voff[lo]).contiguous()
        h1, _, _, _ = ctx.build(k1, 32, v1, o1, hi - lo, hash_keys=True)
        assert h1[0].tobytes() == hh[s].tobytes(), f"segment {s} root differs"
    checked = f"segments {checks} rebuilt alone give the same roots"
    if not args.no_cpu:  # every one of the 100k roots against the independent CPU batch builder
        from oracle import oracle
        tc = time.perf_counter()
        cpu, _ = oracle.batch_roots(keys.cpu().numpy(), (vals[:int(so[-1])].cpu().numpy(), so.astype(np.uint64)),
                                    klen=32, seg_off=offs.astype(np.uint64), hash_keys=True,
                                    nthreads=args.cpu_threads)
        gpu = [hh[s].tobytes() if c[s] else None for s in range(nseg)]
        bad = [s for s in range(nseg) if cpu[s] != gpu[s]]
        assert not bad, f"segmented roots differ from the CPU batch builder: {bad[:5]}"
        checked += f"; all {nseg} roots == the CPU batch builder ({time.perf_counter() - tc:.1f} s)"
    return {"config": f"configs[3]: {nseg} storage tries, {n} slots (log-uniform 1..1e4 per trie)",
            "ms": dt * 1e3, "device_ms": st.t_total_ms, "slots": n, "node_hashes": st.n_node_hashes,
            "node_hashes_per_s": st.n_node_hashes / dt, "node_perms": st.n_node_perms,
            "key_perms": st.n_key_perms, "checked": checked,
            "stage_ms": {"keys": st.t_keys_ms, "sort": st.t_sort_ms, "topology": st.t_topo_ms,
                         "leaves": st.t_leaf_ms, "branches": st.t_branch_ms}}


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--cfg", type=int, nargs="+", default=[2, 4, 3])
    p.add_argument("--steps", type=int, default=5)
    p.add_argument("--warmup", type=int, default=1)
    p.add_argument("--resident", type=int, default=50_000_000)
    p.add_argument("--dirty", type=int, default=20_000, help="configs[2]: dirty accounts per block")
    p.add_argument("--contracts", type=int, default=2_000, help="configs[2]: storage tries (10 dirty slots each)")
    p.add_argument("--no-cpu", action="store_true", help="skip the CPU batch-builder checks")
    p.add_argument("--cpu-threads", type=int, default=16)
    args = p.parse_args()
    for c in args.cfg:
        r = {2: cfg2, 3: cfg3, 4: cfg4}[c](args)
        print(json.dumps(r), flush=True)
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
