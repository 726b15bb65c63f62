"""Secondary workloads of BASELINE.json `configs` on one MI355X (bench.py measures configs[4]).

  --cfg 2  configs[1]: 1M synthetic accounts, full build + root (keys hashed on the GPU).
  --cfg 3  configs[2]: incremental block commit over a resident trie:
           open N_RES accounts (default 50M) with kh_trie_open, then per block 20k dirty
           accounts (90% balance/nonce updates, 5% inserts, 5% deletes) through kh_trie_apply;
           the block's storage side is 2,000 contracts x 1k slots re-rooted as one
           segmented build (kh_dev_trie_build, d_seg), and 50 of them also as resident
           tries with 10 dirty slots each (per-trie kh_trie_apply latency).
  --cfg 4  configs[3]: 100k storage tries, slot counts log-uniform in [1, 1e4], slot key =
           kec256(32-byte BE slot index) (KH_HASH_KEYS), value = RLP(trimmed 1-32 random
           bytes), one segmented build; 4 segments re-built alone must give the same roots.

Inputs are generated on the device before the timed region.  Prints one JSON line per
config.  Parity of these paths is tests/test_gpu_resident.py and test_gpu_parity.py;
here every root is also cross-checked against a from-scratch device build.
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

from khipu_amd import _lib  # noqa: E402
from khipu_amd._lib import KhStats, check, lib  # noqa: E402
from khipu_amd.device import Ctx, ResidentTrie, _ptr  # noqa: E402

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
    ctx = Ctx(0)
    n = args.resident
    g = torch.Generator(device=DEV)
    g.manual_seed(3)
    addr, vals, voff = ctx.synth_accounts(3, 0, n)
    keys = hash_keys(ctx, addr, 20, n)
    del addr
    t = ResidentTrie.__new__(ResidentTrie)
    t.ctx, t.dev, t.h = ctx, DEV, None
    t0 = time.perf_counter()
    t._open(keys, 32, vals, voff, n, False)
    open_s = time.perf_counter() - t0
    del vals, voff
    nupd, nins, ndel = 18_000, 1_000, 1_000
    blocks = []
    for blk in range(args.warmup + args.steps):
        # dirty set: updates/deletes of resident accounts, inserts of fresh addresses
        pick = torch.randperm(n, generator=g, device=DEV)[:nupd + ndel]
        kk = keys[:32 * n].view(n, 32)
        up_old = kk[pick[:nupd]].reshape(-1)
        dels = kk[pick[nupd:]].reshape(-1).clone()
        a2, v2, o2 = ctx.synth_accounts(3, 10**9 + blk * 100_000, nupd + nins)
        new_keys = hash_keys(ctx, a2, 20, nins)[:32 * nins]
        up_keys = torch.cat([up_old, new_keys]).contiguous()
        torch.cuda.synchronize()
        st = KhStats()
        t0 = time.perf_counter()
        root = t.commit_dev(up_keys, v2, o2, nupd + nins, dels, ndel, 32, False, st)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        # later blocks may pick a key deleted earlier: updating it re-inserts it, which
        # is a valid put (the block's dirty set stays 20k records)
        if blk >= args.warmup:
            blocks.append((dt * 1e3, st.t_total_ms, st.n_node_hashes, st.n_leaves))
    live = len(t)
    ms = np.array([b[0] for b in blocks])
    out = {"config": f"configs[2]: 20k dirty accounts per block over a {n // 10**6}M-account resident trie",
           "open_s": open_s, "commit_ms_median": float(np.median(ms)), "commit_ms_all": ms.tolist(),
           "commit_device_ms_median": float(np.median([b[1] for b in blocks])),
           "rehashed_nodes_median": int(np.median([b[2] for b in blocks])), "resident_accounts_after": live,
           "root_after": root.hex()}
    t.close()
    del keys
    torch.cuda.empty_cache()

    # storage side of the block: 2,000 contracts x 1k slots, 10 dirty slots each
    nc, ns = 2000, 1000
    idx = torch.arange(ns, device=DEV, dtype=torch.int64).repeat(nc)
    seg = torch.arange(nc, device=DEV, dtype=torch.int32).repeat_interleave(ns)
    sk = slot_keys(idx)
    sv, so = storage_values(g, nc * ns)
    hh, st = seg_build(ctx, sk, sv, so, seg, nc, nc * ns)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        hh, st = seg_build(ctx, sk, sv, so, seg, nc, nc * ns)
    torch.cuda.synchronize()
    out["storage_segmented_ms"] = (time.perf_counter() - t0) / args.steps * 1e3
    out["storage_segmented"] = f"{nc} storage tries x {ns} slots re-rooted in one segmented build"
    # resident per-contract commits: 10 dirty slots (10% zero = delete) on 50 tries
    lat = []
    skh = sk.view(nc * ns, 32)
    for c in range(50):
        lo, hi = c * ns, (c + 1) * ns
        kc = hash_keys(ctx, skh[lo:hi].reshape(-1).contiguous(), 32, ns)
        vc = sv[int(so[lo]):int(so[hi])].contiguous()
        oc = (so[lo:hi + 1] - so[lo]).contiguous()
        rt = ResidentTrie.__new__(ResidentTrie)
        rt.ctx, rt.dev, rt.h = ctx, DEV, None
        rt._open(kc, 32, vc, oc, ns, False)
        assert rt.root == hh[c].tobytes(), "resident storage root != segmented root"
        kcv = kc[:32 * ns].view(ns, 32)
        up = kcv[0:9].reshape(-1).contiguous()
        uv, uo = storage_values(g, 9)
        dl = kcv[9:10].reshape(-1).contiguous()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        rt.commit_dev(up, uv, uo, 9, dl, 1, 32, False)
        lat.append((time.perf_counter() - t0) * 1e3)
        rt.close()
    out["storage_resident_commit_ms_median"] = float(np.median(lat))
    return out


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
    return {"config": f"configs[3]: {nseg} storage tries, {n} slots (log-uniform 1..1e4 per trie)",
            "ms": dt * 1e3, "device_ms": st.t_total_ms, "slots": n, "node_hashes": st.n_node_hashes,
            "node_hashes_per_s": st.n_node_hashes / dt, "node_perms": st.n_node_perms,
            "key_perms": st.n_key_perms, "checked_segments": checks,
            "stage_ms": {"keys": st.t_keys_ms, "sort": st.t_sort_ms, "topology": st.t_topo_ms,
                         "leaves": st.t_leaf_ms, "branches": st.t_branch_ms}}


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--cfg", type=int, nargs="+", default=[2, 4, 3])
    p.add_argument("--steps", type=int, default=5)
    p.add_argument("--warmup", type=int, default=1)
    p.add_argument("--resident", type=int, default=50_000_000)
    args = p.parse_args()
    for c in args.cfg:
        r = {2: cfg2, 3: cfg3, 4: cfg4}[c](args)
        print(json.dumps(r), flush=True)
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
