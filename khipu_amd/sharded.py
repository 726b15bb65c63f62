"""Multi-GPU state root: the trie sharded by top key nibble over one process per GPU.

SURVEY §8(e).  Rank r of N owns top nibbles q with q * N // 16 == r (2 per GPU at
N = 8).  One step, from (address, account body) records spread over the ranks:

  1. kec256 of the local addresses                         (libkhst, k_hash_keys)
  2. stable partition of the local records by owner rank   (libkhst, kh_dev_partition_ev:
     the value bytes are still being copied while the keys are exchanged)
  3. exchange: all-to-all of counts, keys, value lengths and value bytes
     (torch.distributed = RCCL over xGMI; rank-major order keeps "later put wins")
  4. build the owned subtries from nibble 1 down           (libkhst, depth0 = 1)
  5. all-gather the 16 capped references, fold into the root branch on the host
     (kh_fold_root16; MerklePatriciaTrie.scala:169 — the root is always hashed)

If fewer than two top nibbles are occupied the root is not a branch: the owner of
the single occupied nibble holds every key and builds the whole trie (depth0 = 0).

The communication code is backend-agnostic: GpuBackend runs libkhst on the
rank's GPU with NCCL(RCCL) tensors; tests use a CPU backend with gloo.
"""
import numpy as np
import torch
import torch.distributed as dist

REF_BYTES = 32 + 32 + 8  # hash | inline encoding | length (LE u64)


def owner_of_nibble(q, world):
    return (q * world) >> 4


class GpuBackend:
    """libkhst.so on the rank's GPU; tensors live in HBM (torch is the allocator)."""

    def __init__(self, device):
        from .device import Ctx
        self.ctx = Ctx(device)
        self.device = torch.device(f"cuda:{device}")
        self.last_stats = None
        self.overlap = True  # value exchange beside the key sort / topology (exchange())

    def hash_keys(self, addr, n, klen=20):
        from ._lib import check, lib
        from .device import _ptr
        out = torch.empty(n * 32 + 64, dtype=torch.uint8, device=self.device)
        torch.cuda.synchronize(self.device)
        check(lib().kh_dev_hash_keys(self.ctx.h, _ptr(addr), klen, n, _ptr(out)))
        return out

    def partition(self, keys32, vals, voff, n, nparts):
        """With self.overlap the value bytes are still being copied on return (the keys,
        lengths and counts are in place): self.vals_done is the event after them, which
        exchange() orders the value all-to-all after (kh_dev_partition_ev)."""
        from ._lib import check, lib
        from .device import _ptr
        pk = torch.empty(n * 32 + 64, dtype=torch.uint8, device=self.device)
        pv = torch.empty(vals.numel() + 64, dtype=torch.uint8, device=self.device)
        pl = torch.empty(max(n, 1), dtype=torch.int64, device=self.device)
        cnt = np.zeros(16, np.uint64)
        nb = np.zeros(16, np.uint64)
        torch.cuda.synchronize(self.device)
        self.vals_done = None
        ev = None
        if self.overlap:
            self.vals_done = torch.cuda.Event()
            self.vals_done.record()  # creates the event; the library records it again on its stream
            ev = self.vals_done.cuda_event
        check(lib().kh_dev_partition_ev(self.ctx.h, ev, _ptr(keys32), _ptr(vals), _ptr(voff), n, nparts, _ptr(pk),
                                        _ptr(pv), _ptr(pl), cnt.ctypes.data, nb.ctypes.data))
        return pk, pv, pl, cnt[:nparts].astype(np.int64), nb[:nparts].astype(np.int64)

    def hash_partition(self, addr, vals, voff, n, nparts, klen=20):
        """hash_keys + partition in one library call (kh_dev_hash_partition_ev: the hashing
        pass writes each key's owner as a byte, which the count pass reads instead of the
        keys' lines); same outputs and overlap as partition().  What the step runs at N > 1
        (scripts/shard_rank_sim.py times both forms)."""
        from ._lib import check, lib
        from .device import _ptr
        pk = torch.empty(n * 32 + 64, dtype=torch.uint8, device=self.device)
        pv = torch.empty(vals.numel() + 64, dtype=torch.uint8, device=self.device)
        pl = torch.empty(max(n, 1), dtype=torch.int64, device=self.device)
        cnt = np.zeros(16, np.uint64)
        nb = np.zeros(16, np.uint64)
        torch.cuda.synchronize(self.device)
        self.vals_done = None
        ev = None
        if self.overlap:
            self.vals_done = torch.cuda.Event()
            self.vals_done.record()  # creates the event; the library records it again on its stream
            ev = self.vals_done.cuda_event
        check(lib().kh_dev_hash_partition_ev(self.ctx.h, ev, _ptr(addr), klen, _ptr(vals), _ptr(voff), n, nparts,
                                             _ptr(pk), _ptr(pv), _ptr(pl), cnt.ctypes.data, nb.ctypes.data))
        return pk, pv, pl, cnt[:nparts].astype(np.int64), nb[:nparts].astype(np.int64)

    def wait(self, ev):
        """The current (torch) stream waits for ev; the host does not."""
        torch.cuda.current_stream(self.device).wait_event(ev)

    def build(self, keys32, vals, voff, n, depth0, vals_ready=None):
        """vals_ready: a torch.cuda.Event after which vals / voff are in place (the keys
        must be in place already); the sort and the topology do not wait for it."""
        hh, ll, ii, st = self.ctx.build(keys32, 32, vals, voff, n, depth0=depth0, vals_ready=vals_ready)
        self.last_stats = st
        return hh, ll, ii

    def event(self):
        """An event on the current (torch) stream: everything enqueued so far."""
        e = torch.cuda.Event()
        e.record()
        return e

    def fold(self, hh, ll, ii):
        from .device import fold_root16
        return fold_root16(hh, ll, ii)

    def empty(self, nbytes, dtype=torch.uint8):
        return torch.empty(nbytes, dtype=dtype, device=self.device)

    def sync(self):
        torch.cuda.synchronize(self.device)


A2A_CHUNK = 1 << 30  # bytes per peer per all-to-all round (keeps every count < 2^31)


def a2a_rounds(biggest, chunk=None):
    """Rounds a2a_bytes needs for a largest per-peer split of `biggest` bytes over all
    ranks (every rank must run the same number)."""
    return int(-(-int(biggest) // (chunk or A2A_CHUNK)))


def a2a_bytes(out, inp, out_splits, in_splits, rounds, chunk=None, async_op=False):
    """all_to_all_single of uint8 buffers with per-peer byte splits, in `rounds` rounds
    of at most `chunk` bytes per peer so no message count reaches 2^31 (RCCL / c10d
    take int counts).  async_op: returns the works to wait on (single-round only; the
    multi-round path copies between rounds and so runs synchronously)."""
    world = len(in_splits)
    chunk = chunk or A2A_CHUNK
    if rounds <= 1:
        w = dist.all_to_all_single(out, inp, list(out_splits), list(in_splits), async_op=async_op)
        return [w] if async_op else []
    ioff = np.concatenate([[0], np.cumsum(in_splits)])
    ooff = np.concatenate([[0], np.cumsum(out_splits)])
    for r in range(rounds):
        lo = r * chunk
        isz = [int(max(0, min(chunk, in_splits[p] - lo))) for p in range(world)]
        osz = [int(max(0, min(chunk, out_splits[p] - lo))) for p in range(world)]
        send = torch.cat([inp[int(ioff[p]) + lo:int(ioff[p]) + lo + isz[p]] for p in range(world)])
        recv = torch.empty(sum(osz), dtype=inp.dtype, device=inp.device)
        dist.all_to_all_single(recv, send, osz, isz)
        o = 0
        for p in range(world):
            out[int(ooff[p]) + lo:int(ooff[p]) + lo + osz[p]].copy_(recv[o:o + osz[p]])
            o += osz[p]
    return []


def exchange(be, pkeys, pvals, pvlen, counts, nbytes):
    """All-to-all of the partitioned records.  Returns (keys32, vals, voff, m, vals_ready)
    of the records this rank owns, ordered by source rank then source order.  The keys
    are in place on return; the value lengths and bytes may still be in flight:
    vals_ready (a device event, or None when everything has landed) orders the build's
    value reads after them, so the key sort and the topology overlap the larger
    transfer."""
    world = dist.get_world_size()
    dev = pkeys.device
    # counts and byte counts in one all-to-all: rank p receives (counts[p], nbytes[p]) pairs
    send = torch.tensor(np.stack([counts, nbytes], 1).reshape(-1).astype(np.int64), device=dev)
    recv = torch.empty_like(send)
    dist.all_to_all_single(recv, send, [2] * world, [2] * world)
    rr = recv.cpu().numpy().reshape(world, 2)
    rc, rb = rr[:, 0].astype(np.int64), rr[:, 1].astype(np.int64)
    m = int(rc.sum())
    tot_b = int(rb.sum())
    cl, bl = [int(x) for x in counts], [int(x) for x in nbytes]
    n_send, b_send = sum(cl), sum(bl)
    # every rank runs the same number of rounds per transfer: agree on the largest splits
    big = torch.tensor([max(cl + [int(c) for c in rc] + [0]) * 32, max(bl + [int(b) for b in rb] + [0])],
                       dtype=torch.int64, device=dev)
    dist.all_reduce(big, op=dist.ReduceOp.MAX)
    kr, vr = (a2a_rounds(x) for x in big.cpu().tolist())
    rkeys = be.empty(m * 32 + 64)
    a2a_bytes(rkeys[:m * 32], pkeys[:n_send * 32], [int(c) * 32 for c in rc], [c * 32 for c in cl], kr)
    keys_done = be.event() if be.overlap else None
    rlen = be.empty(max(m, 1), torch.int64)
    rvals = be.empty(tot_b + 64)
    works = a2a_bytes(rlen[:m].view(torch.uint8), pvlen[:n_send].view(torch.uint8), [int(c) * 8 for c in rc],
                      [c * 8 for c in cl], kr, async_op=be.overlap)
    vals_done = getattr(be, "vals_done", None)  # the partition's value copy may still be running
    if vals_done is not None:
        be.wait(vals_done)
    works += a2a_bytes(rvals[:tot_b], pvals[:b_send], [int(b) for b in rb], bl, vr, async_op=be.overlap)
    for w in works:
        w.wait()  # the current stream waits; the host does not
    voff = torch.zeros(m + 1, dtype=torch.int64, device=dev)
    if m:
        torch.cumsum(rlen[:m], 0, out=voff[1:])
    if keys_done is None:
        return rkeys, rvals, voff, m, None
    vals_ready = be.event()
    keys_done.synchronize()  # the keys have landed (the values may not have)
    return rkeys, rvals, voff, m, vals_ready


def gather_refs(be, hh, ll, ii):
    """All-gather the 16 subtrie references of every rank; each nibble's reference is
    taken from its owner."""
    world, rank = dist.get_world_size(), dist.get_rank()
    buf = np.zeros((16, REF_BYTES), np.uint8)
    buf[:, :32] = hh
    buf[:, 32:64] = ii
    buf[:, 64:72] = ll.astype(np.uint64).view(np.uint8).reshape(16, 8)
    mine = torch.from_numpy(buf.reshape(-1).copy()).to(be.empty(1).device)
    allb = be.empty(world * 16 * REF_BYTES)
    dist.all_gather_into_tensor(allb, mine)
    a = allb.cpu().numpy().reshape(world, 16, REF_BYTES)
    H = np.zeros((16, 32), np.uint8)
    I = np.zeros((16, 32), np.uint8)
    L = np.zeros(16, np.uint32)
    for q in range(16):
        o = owner_of_nibble(q, world)
        H[q] = a[o, q, :32]
        I[q] = a[o, q, 32:64]
        L[q] = int(a[o, q, 64:72].view(np.uint64)[0])
    return H, L, I


def sharded_root(be, addr, vals, voff, n, klen=20, keys_prehashed=False, phases=None):
    """One sharded state-root step.  Every rank calls it with its slice of the records;
    every rank returns the root (bytes) and the number of node hashes it computed.
    phases: optional dict that receives each phase's wall time in ms (synchronising
    the device after every phase: a diagnostic run, not the timed one)."""
    import time
    world = dist.get_world_size()
    t = [time.perf_counter()]

    def mark():
        if phases is not None:
            be.sync()
            t.append(time.perf_counter())

    if world == 1:  # nothing to route: the build reads the records where they are
        keys32 = addr if keys_prehashed else be.hash_keys(addr, n, klen)
        mark()
        rk, rv, ro, m, ready = keys32, vals, voff, n, None
        mark()
        mark()
    else:
        if keys_prehashed:
            mark()
            pk, pv, pl, cnt, nb = be.partition(addr, vals, voff, n, world)
        else:
            # hashing and partition in one call (kh_dev_hash_partition_ev: the hashing pass
            # writes each key's owner byte, the count pass reads those instead of the keys;
            # profiles/r4aw_hash_partition_ab_world8.json)
            pk, pv, pl, cnt, nb = be.hash_partition(addr, vals, voff, n, world, klen)
            mark()
        mark()
        rk, rv, ro, m, ready = exchange(be, pk, pv, pl, cnt, nb)
        mark()
    hh, ll, ii = be.build(rk, rv, ro, m, depth0=1, vals_ready=None if phases is not None else ready)
    mark()
    H, L, I = gather_refs(be, hh, ll, ii)
    mark()
    if phases is not None:
        for name, a, b in zip(("hash_keys", "partition", "exchange", "build", "gather"), t, t[1:]):
            phases[name] = (b - a) * 1e3
    occupied = [q for q in range(16) if L[q] > 0]
    if len(occupied) >= 2:
        return be.fold(H, L, I)
    # root is not a branch: the owner of the one occupied nibble has every key
    from .trie import EMPTY_TRIE_HASH
    if not occupied:
        return EMPTY_TRIE_HASH
    o = owner_of_nibble(occupied[0], world)
    root = torch.zeros(32, dtype=torch.uint8, device=be.empty(1).device)
    if dist.get_rank() == o:
        h, _, _ = be.build(rk, rv, ro, m, depth0=0)
        root.copy_(torch.from_numpy(h[0].copy()))
    dist.broadcast(root, o)
    return root.cpu().numpy().tobytes()


# State roots of the synthetic workloads (csrc/synth.h), keyed by (config id, accounts),
# each asserted equal to the independent CPU batch builder (oracle/batch_root.cc) by a
# full-size `bench.py` run (profiles/r2zp_bench_100m.json, profiles/r3a_bench_100m.json).
PINNED_ROOTS = {
    (5, 100_000_000): "577f095224664dc395ca23578afe7bd0c82dbeb5a863285af99e8271a81b9cad",
}


def self_check(be, cfg, n_total, root):
    """Rank 0: the sharded root must equal the single-GPU root of the SAME workload
    (regenerated in full on this rank: the synthesis is counter-based) and, where one is
    pinned, the CPU-checked root.  Returns (ok, report)."""
    import torch as _t
    A, V, O = be.ctx.synth_accounts(cfg, 0, n_total)
    hh, _, _, _ = be.ctx.build(A, 20, V, O, n_total, hash_keys=True)
    single = hh[0].tobytes()
    del A, V, O
    _t.cuda.empty_cache()
    pinned = PINNED_ROOTS.get((cfg, n_total))
    ok = single == root and (pinned is None or pinned == root.hex())
    return ok, {"single_gpu_root": single.hex(), "pinned_root": pinned,
                "sharded_root_equal": ok}


def bench_main(args):
    """bench.py --gpus N under torch.distributed.run: strong scaling of the fixed
    args.accounts trie over WORLD_SIZE GPUs (one rank per GPU, RCCL)."""
    import json
    import os
    import time
    if "RANK" not in os.environ:  # `bench.py --sharded` without a launcher: a world of one
        import socket
        with socket.socket() as s:
            s.bind(("127.0.0.1", 0))
            port = s.getsockname()[1]
        os.environ.update(RANK="0", WORLD_SIZE="1", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dist.init_process_group("nccl", device_id=torch.device(f"cuda:{local}"))
    be = GpuBackend(local)
    n_total = args.accounts
    first = n_total * rank // world
    n = n_total * (rank + 1) // world - first
    addr, vals, voff = be.ctx.synth_accounts(args.cfg, first, n)
    be.sync()

    def step():
        return sharded_root(be, addr, vals, voff, n)

    for _ in range(args.warmup):
        step()
    be.sync()
    dist.barrier()
    be.sync()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        root = step()
    be.sync()
    dist.barrier()
    be.sync()
    dt = torch.tensor([(time.perf_counter() - t0) / args.steps], dtype=torch.float64, device=f"cuda:{local}")
    dist.all_reduce(dt, op=dist.ReduceOp.MAX)
    st = be.last_stats
    hashes = torch.tensor([st.n_node_hashes, st.n_leaves, st.n_branches], dtype=torch.int64, device=f"cuda:{local}")
    dist.all_reduce(hashes)
    dt = float(dt.item())
    node_hashes = int(hashes[0].item()) + 1  # + the folded root branch
    # roofline of the dominant kernel (k_leaf_in, one launch per rank per step), on the
    # slowest rank: its HIP-event time on the library's stream
    leaf = torch.tensor([st.t_leaf_ms, float(st.n_leaves)], dtype=torch.float64, device=f"cuda:{local}")
    leaf_all = [torch.zeros_like(leaf) for _ in range(world)]
    dist.all_gather(leaf_all, leaf)
    leaf_all = [x.tolist() for x in leaf_all]
    slow = max(leaf_all, key=lambda x: x[0])
    VALU_PEAK, OPS = 256 * 4 * 32 * 2.4e9, 5760
    achieved = slow[1] * OPS / max(slow[0] * 1e-3, 1e-12)
    import bench
    roof = {"kernel": "k_leaf_in", "bound": "valu", "achieved": achieved / 1e12, "peak": VALU_PEAK / 1e12,
            "unit": "T int32-lane-ops/s", "frac": achieved / VALU_PEAK,
            "traffic": bench.pmc_traffic_per_unit("k_leaf_in", slow[1]),
            "traffic_note": "HBM bytes per launch: the committed 100M PMC summary's bytes per leaf x this launch's leaves",
            "avg_ms": slow[0], "perms_per_launch": int(slow[1]), "rank": "slowest of the ranks"}
    # one more (untimed) step with a device sync after every phase: where the time goes
    phases = {}
    sharded_root(be, addr, vals, voff, n, phases=phases)
    ph = torch.tensor([phases[k] for k in sorted(phases)], dtype=torch.float64, device=f"cuda:{local}")
    dist.all_reduce(ph, op=dist.ReduceOp.MAX)
    phases = {k: round(float(v), 3) for k, v in zip(sorted(phases), ph.tolist())}
    # self-check (after the timed region): a wrong root must not be reported as throughput
    ok = torch.ones(1, dtype=torch.int64, device=f"cuda:{local}")
    check = None
    if rank == 0:
        good, check = self_check(be, args.cfg, n_total, root)
        ok[0] = int(good)
    dist.broadcast(ok, 0)
    if not int(ok.item()):
        if rank == 0:
            import sys
            print(f"sharded root {root.hex()} FAILED its self-check: {check}", file=sys.stderr, flush=True)
        dist.barrier()
        dist.destroy_process_group()
        raise SystemExit(1)
    if rank == 0:
        out = {
            "metric": "node-hashes/sec (full state root, 100M-account trie)",
            "value": node_hashes / dt, "unit": "node-hashes/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": dt * 1e3, "higher_is_better": True, "scaling": "strong",
            "vs_baseline": None, "dtype": "u64",
            "data": "synthetic (counter-based accounts, SURVEY §8d, csrc/synth.h)",
            "config": {"workload": f"{n_total} synthetic accounts -> state root, sharded by top key nibble",
                       "accounts": n_total, "parallelism": f"nibble-shard x{world} (RCCL all-to-all + gather)"},
            "state_root": root.hex(),
            "topology": {"n_leaves": int(hashes[1].item()), "n_branches": int(hashes[2].item()) + 1,
                         "n_node_hashes": node_hashes},
            "parity": check,
            "phase_ms_max_over_ranks": phases,
            "per_rank_build_ms": st.t_total_ms,
            "roofline": roof,
        }
        if not getattr(args, "no_cpu", False):
            # the khipu-faithful sequential CPU trie is timed at N = 1 only (rank 0; its 4-sample
            # fit up to 1M accounts, each sample's root asserted against the GPU's); an N > 1 line
            # reports the newest committed N = 1 measurement, named by its file.  A world-1 run of
            # this path (no committed line) times the small samples itself.
            cb = bench.committed_cpu_baseline() if world > 1 else None
            if cb is None:
                samples = [int(x) for x in str(getattr(args, "seq_samples", "20000,50000")).split(",")
                           if x and int(x) <= min(n, 50_000)]
                cb = bench.cpu_baseline(be.ctx, args.cfg, addr, vals, voff, samples) if samples else None
            if cb:
                out["cpu_baseline"] = cb
        print(json.dumps(out), flush=True)
    dist.barrier()
    dist.destroy_process_group()
