"""configs[2] block workload, shared by tests/test_gpu_configs.py
(1M resident accounts, checked against the CPU batch builder and the oracle) and
scripts/bench_configs.py (50M resident accounts).  Test / bench infrastructure only.

State: n synthetic accounts (csrc/synth.h, config 3) in a resident state trie (32-byte
keys = kec256(address), computed on the device); the first `nc` accounts are contracts
owning resident storage tries of `ns` slots each, all in one forest (trie id = contract
index; slot key = kec256(32-byte big-endian slot index), KH_HASH_KEYS; value =
RLP(trimmed 1-32 random bytes)).  A setup block loads every slot and writes the storage
roots into the contract bodies.

Block b (one kh_block_commit): `dirty` account ops = 90% updates (the nc contracts, whose
storage changes, plus random other accounts), 5% inserts of fresh addresses, 5% deletes;
per contract 10 dirty slots: 8 updates, 1 insert, 1 delete (a zero value,
TrieStorage.scala:44-46).  Storage roots first, then the account leaves
(BlockWorldState.scala:243-252).

Deleted accounts come from the tail [n - nblocks * ndel, n) and deleted slots from the
per-trie range [ns - nblocks, ns); neither is upserted again, so the final state is
(initial records minus those ranges) followed by every block's upserts in order -- one
plain build of that sequence (later puts win) must give the same roots.
"""
import numpy as np
import torch

from khipu_amd import _lib
from khipu_amd._lib import KhStats, check, lib
from khipu_amd.device import ResidentForest, ResidentTrie, _ptr, block_commit

CFG = 3


def hash_keys(ctx, d_in, klen, n):
    out = torch.empty(n * 32 + 64, dtype=torch.uint8, device=d_in.device)
    torch.cuda.synchronize()
    check(lib().kh_dev_hash_keys(ctx.h, _ptr(d_in), klen, n, _ptr(out)))
    torch.cuda.synchronize()
    return out[:32 * n]


def storage_values(g, n, dev):
    """RLP(trimmed 1-32 random bytes) per slot (rlpDataWordSerializer, trie/package.scala:28-32)."""
    L = torch.randint(1, 33, (n,), generator=g, device=dev)
    b0 = torch.randint(1, 256, (n,), generator=g, device=dev)
    raw = (L == 1) & (b0 < 0x80)
    elen = torch.where(raw, 1, L + 1)
    voff = torch.zeros(n + 1, dtype=torch.int64, device=dev)
    voff[1:] = torch.cumsum(elen, 0)
    vals = torch.randint(0, 256, (int(voff[-1]) + 64,), generator=g, device=dev, dtype=torch.uint8)
    st = voff[:-1]
    pre = ~raw
    vals[st[pre]] = (0x80 + L[pre]).to(torch.uint8)
    vals[st + pre.long()] = b0.to(torch.uint8)
    return vals, voff


def slot_keys(idx):
    """32-byte big-endian slot indices (DataWord; hashed by hashDataWordSerializable)."""
    k = torch.zeros(idx.numel(), 32, dtype=torch.uint8, device=idx.device)
    for b in range(8):
        k[:, 31 - b] = ((idx >> (8 * b)) & 0xFF).to(torch.uint8)
    return k.reshape(-1)


def spans(vals, voff, idx):
    """Packed copy of the value spans idx (device)."""
    lens = voff[idx + 1] - voff[idx]
    off = torch.zeros(idx.numel() + 1, dtype=torch.int64, device=vals.device)
    off[1:] = torch.cumsum(lens, 0)
    tot = int(off[-1])
    src = torch.repeat_interleave(voff[idx] - off[:-1], lens) + torch.arange(tot, device=vals.device)
    out = torch.zeros(tot + 64, dtype=torch.uint8, device=vals.device)
    out[:tot] = vals[src]
    return out, off


class BlockWorkload:
    def __init__(self, ctx, n, nblocks, seed=3, nc=2000, ns=1000, dirty=20_000, emit=False):
        self.ctx, self.n, self.nblocks, self.nc, self.ns = ctx, n, nblocks, nc, ns
        self.dev = f"cuda:{ctx.device}"
        self.g = torch.Generator(device=self.dev)
        self.g.manual_seed(seed)
        self.nins = self.ndel = dirty // 20
        self.nupd = dirty - self.nins - self.ndel
        assert self.nupd > nc and n > nc + nblocks * self.ndel + self.nupd
        addr, self.vals, self.voff = ctx.synth_accounts(CFG, 0, n)
        self.keys = hash_keys(ctx, addr, 20, n)
        del addr
        self.state = ResidentTrie.__new__(ResidentTrie)
        self.state.ctx, self.state.dev, self.state.h = ctx, self.dev, None
        self.state._open(self.keys, 32, self.vals, self.voff, n, False, emit=emit)
        self.forest = ResidentForest(ctx, hash_keys=True, emit=emit)
        self.ups = []        # every block's account upserts (keys, bodies, offsets) in order
        self.ups_pristine = []  # the same bodies as handed in, before kh_block_commit patched
                                # the contracts' stateRoot fields in place
        self.slot_ups = []   # every block's storage upserts (trie, slot keys, values, offsets)
        self.roots = {}      # last root per storage trie
        self.t_commit = []
        # setup block: every slot, and the contract bodies with their storage roots
        tid = torch.arange(nc, device=self.dev, dtype=torch.int32).repeat_interleave(ns)
        sk = slot_keys(torch.arange(ns, device=self.dev, dtype=torch.int64).repeat(nc))
        sv, so = storage_values(self.g, nc * ns, self.dev)
        ck = self.keys[:32 * nc].clone()
        cv, co = spans(self.vals, self.voff, torch.arange(nc, device=self.dev))
        self._commit(tid, sk, sv, so, None, None, ck, cv, co, torch.arange(nc, device=self.dev, dtype=torch.int32),
                     None, timed=False)

    def _commit(self, s_tid, s_keys, s_vals, s_voff, d_tid, d_keys, a_keys, a_vals, a_voff, a_tid, a_del, timed=True):
        ns_up = s_tid.numel()
        ns_del = 0 if d_tid is None else d_tid.numel()
        na_up = a_tid.numel()
        na_del = 0 if a_del is None else a_del.numel() // 32
        st = KhStats()
        self.ups_pristine.append(a_vals.clone())
        torch.cuda.synchronize()
        import time
        t0 = time.perf_counter()
        root = block_commit(self.state, self.forest, s_tid, s_keys, s_vals, s_voff, ns_up, d_tid, d_keys, ns_del,
                            a_keys, a_vals, a_voff, a_tid, na_up, a_del, na_del, stats=st)
        torch.cuda.synchronize()
        if timed:
            self.t_commit.append(((time.perf_counter() - t0) * 1e3, st.n_node_hashes, st.n_inputs))
        self.ups.append((a_keys, a_vals, a_voff, na_up))
        self.slot_ups.append((s_tid, s_keys, s_vals, s_voff))
        self.roots.update(self.forest.last_roots())
        return root

    def block(self, b):
        """One block's ops (device tensors) and its kh_block_commit; returns the state root."""
        return self._commit(*self.prepare(b))

    def commit_prepared(self, ops):
        """kh_block_commit of ops made by prepare(b) (profiling: inputs made beforehand)."""
        return self._commit(*ops)

    def prepare(self, b):
        """Block b's ops as device tensors (the arguments of _commit)."""
        nc, ns, dev, g = self.nc, self.ns, self.dev, self.g
        D = self.nblocks * self.ndel
        pool = torch.randperm(self.n - D - nc, generator=g, device=dev)[:self.nupd - nc] + nc
        upd_idx = torch.cat([torch.arange(nc, device=dev), pool])
        _, ub, uo = self.ctx.synth_accounts(CFG, 2 * 10**9 + b * 100_000, self.nupd)  # new bodies
        a2, ib, io = self.ctx.synth_accounts(CFG, 10**9 + b * 100_000, self.nins)     # fresh accounts
        ins_keys = hash_keys(self.ctx, a2, 20, self.nins)
        kk = self.keys.view(self.n, 32)
        a_keys = torch.cat([kk[upd_idx].reshape(-1), ins_keys]).contiguous()
        ub_n, ib_n = int(uo[-1]), int(io[-1])
        a_vals = torch.zeros(ub_n + ib_n + 64, dtype=torch.uint8, device=dev)
        a_vals[:ub_n] = ub[:ub_n]
        a_vals[ub_n:ub_n + ib_n] = ib[:ib_n]
        a_voff = torch.cat([uo, io[1:] + ub_n]).contiguous()
        a_tid = torch.full((self.nupd + self.nins,), _lib.KH_NO_TRIE, dtype=torch.int64, device=dev)
        a_tid[:nc] = torch.arange(nc, device=dev)
        a_tid = a_tid.to(torch.int32)
        lo = self.n - D + b * self.ndel
        a_del = kk[lo:lo + self.ndel].reshape(-1).contiguous()
        # storage: per contract 8 updates of live slots, 1 new slot, 1 delete
        upd_slot = torch.randint(0, ns - self.nblocks, (nc, 8), generator=g, device=dev)
        new_slot = torch.full((nc, 1), ns + b, device=dev, dtype=torch.int64)
        s_idx = torch.cat([upd_slot, new_slot], 1).reshape(-1)
        s_tid = torch.arange(nc, device=dev, dtype=torch.int32).repeat_interleave(9)
        s_keys = slot_keys(s_idx)
        s_vals, s_voff = storage_values(g, nc * 9, dev)
        d_tid = torch.arange(nc, device=dev, dtype=torch.int32)
        d_keys = slot_keys(torch.full((nc,), ns - 1 - b, device=dev, dtype=torch.int64))
        return (s_tid, s_keys, s_vals, s_voff, d_tid, d_keys, a_keys, a_vals, a_voff, a_tid, a_del)

    # ---- verification: one plain build of the final sequence of puts
    def final_accounts(self, bodies=None):
        """(keys, vals, voff, N) device tensors: the initial records minus the deleted tail,
        then every block's upserts in order (later puts win).  bodies: optional list of
        per-block body buffers replacing the committed ones (same offsets)."""
        m = self.n - self.nblocks * self.ndel
        parts_k = [self.keys[:32 * m]]
        v0 = int(self.voff[m])
        parts_v = [self.vals[:v0]]
        parts_o = [self.voff[:m]]
        base = v0
        for bi, (k, v, o, cnt) in enumerate(self.ups):
            if bodies is not None:
                v = bodies[bi]
            parts_k.append(k[:32 * cnt])
            parts_v.append(v[:int(o[cnt])])
            parts_o.append(o[:cnt] + base)
            base += int(o[cnt])
        keys = torch.cat(parts_k).contiguous()
        vals = torch.cat(parts_v + [torch.zeros(64, dtype=torch.uint8, device=self.dev)]).contiguous()
        N = keys.numel() // 32
        voff = torch.cat(parts_o + [torch.tensor([base], device=self.dev)]).contiguous()
        return keys, vals, voff, N

    def final_storage(self):
        """(slot keys, vals, voff, trie ids, N) of every storage trie's final slot set: the
        setup slots minus the deleted range, then every block's upserts in order."""
        s_tid, s_keys, s_vals, s_voff = self.slot_ups[0]
        nc, ns = self.nc, self.ns
        keep = (torch.arange(nc * ns, device=self.dev) % ns) < (ns - self.nblocks)
        idx = torch.nonzero(keep).flatten()
        kv, ko = spans(s_vals, s_voff, idx)
        tids = [s_tid[idx]]
        keys = [s_keys.view(-1, 32)[idx].reshape(-1)]
        vals = [kv[:int(ko[-1])]]
        offs = [ko[:-1]]
        base = int(ko[-1])
        for t, k, v, o in self.slot_ups[1:]:
            cnt = t.numel()
            tids.append(t)
            keys.append(k[:32 * cnt])
            vals.append(v[:int(o[cnt])])
            offs.append(o[:cnt] + base)
            base += int(o[cnt])
        tid = torch.cat(tids)
        order = torch.sort(tid.to(torch.int64), stable=True).indices  # segments contiguous, put order kept
        K = torch.cat(keys).view(-1, 32)[order].reshape(-1).contiguous()
        V = torch.cat(vals)
        O = torch.cat(offs + [torch.tensor([base], device=self.dev)])
        Vs, Os = spans(V, O, order)
        return K, Vs, Os, tid[order].contiguous(), order.numel()
