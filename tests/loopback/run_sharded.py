"""TEST INFRASTRUCTURE ONLY: runs kh_trie_root_sharded's RCCL branch (csrc/sharded.h) through
the in-process loopback RCCL (tests/loopback/librccl.so) on the box's one GPU.  A process of
its own: the loopback must be loaded (RTLD_GLOBAL, soname librccl.so) before the library's
first sharded call resolves RCCL, and that resolution holds for the process.

    python tests/loopback/run_sharded.py CASES.npz [--full]

CASES.npz (written by tests/test_gpu_loopback_rccl.py): for case i, keys_i (n x klen uint8),
vals_i (uint8), voff_i (uint64), meta_i = [klen, hash_keys, world].  Prints one JSON line per
case: the root over the loopback exchange (KH_SHARD_RCCL), the root over the device-copy
exchange, the single-GPU root, and the loopback's matched operations / bytes for the call.
--full adds the configs[4] workload (100M synthetic accounts, eight owner shards)."""
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def main():
    lb = ctypes.CDLL(os.path.join(ROOT, "tests", "loopback", "librccl.so"), mode=ctypes.RTLD_GLOBAL)
    import numpy as np
    from khipu_amd import trie

    def stats():
        o, b, g = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_uint64()
        lb.loopback_stats(ctypes.byref(o), ctypes.byref(b), ctypes.byref(g))
        return o.value, b.value, g.value

    d = np.load(sys.argv[1])
    i = 0
    while f"meta_{i}" in d:
        klen, hk, world = (int(x) for x in d[f"meta_{i}"])
        keys, vals, voff = d[f"keys_{i}"], d[f"vals_{i}"], d[f"voff_{i}"].astype(np.uint64)
        o0, b0, _ = stats()
        rl = trie.trie_root_sharded(keys, (vals, voff), [0] * world, hash_keys=bool(hk), klen=klen, rccl=True)
        o1, b1, _ = stats()
        rc = trie.trie_root_sharded(keys, (vals, voff), [0] * world, hash_keys=bool(hk), klen=klen)
        o2, _, _ = stats()
        r1 = trie.trie_root(keys, (vals, voff), hash_keys=bool(hk), klen=klen)
        print(json.dumps({"case": i, "loopback": rl.hex(), "copies": rc.hex(), "single": r1.hex(),
                          "ops": o1 - o0, "bytes": b1 - b0, "ops_copy_path": o2 - o1}), flush=True)
        i += 1
    if "--full" in sys.argv:
        # (no torch in this process: torch's libtorch_hip would bind its RCCL symbols to the
        # loopback loaded above; the workload is made by the library's synth kernel into hipMalloc'd
        # buffers and copied to host memory, 10M accounts at a time)
        from khipu_amd import lib as khlib
        hip = ctypes.CDLL("libamdhip64.so")
        n, cfg, chunk = 100_000_000, 5, 10_000_000
        pinned = "577f095224664dc395ca23578afe7bd0c82dbeb5a863285af99e8271a81b9cad"  # khipu_amd.sharded.PINNED_ROOTS
        L = khlib()
        ctx = ctypes.c_void_p()
        assert L.kh_ctx_create(0, ctypes.byref(ctx)) == 0
        bufs = [ctypes.c_void_p() for _ in range(3)]
        sizes = [chunk * 20 + 64, chunk * 96 + 64, (chunk + 1) * 8]
        for b, sz in zip(bufs, sizes):
            assert hip.hipMalloc(ctypes.byref(b), ctypes.c_size_t(sz)) == 0
        a = np.empty(n * 20, np.uint8)
        vb = np.empty(n * 96, np.uint8)
        vo = np.zeros(n + 1, np.uint64)
        tot = 0
        for f in range(0, n, chunk):
            assert L.kh_dev_synth_accounts(ctx, cfg, f, chunk, bufs[0], bufs[1], bufs[2]) == 0
            assert hip.hipDeviceSynchronize() == 0
            off = np.empty(chunk + 1, np.uint64)
            assert hip.hipMemcpy(off.ctypes.data_as(ctypes.c_void_p), bufs[2], ctypes.c_size_t(off.nbytes), 2) == 0
            nb = int(off[-1])
            assert hip.hipMemcpy(ctypes.c_void_p(a.ctypes.data + 20 * f), bufs[0], ctypes.c_size_t(20 * chunk), 2) == 0
            assert hip.hipMemcpy(ctypes.c_void_p(vb.ctypes.data + tot), bufs[1], ctypes.c_size_t(nb), 2) == 0
            vo[f:f + chunk + 1] = off + np.uint64(tot)
            tot += nb
        for b in bufs:
            hip.hipFree(b)
        L.kh_ctx_destroy(ctx)
        o0, b0, g0 = stats()
        t0 = time.perf_counter()
        r = trie.trie_root_sharded(a, (vb[:tot], vo), [0] * 8, hash_keys=True, klen=20, rccl=True)
        t = time.perf_counter() - t0
        o1, b1, g1 = stats()
        print(json.dumps({"case": "config4_100m", "loopback": r.hex(), "pinned": pinned,
                          "ops": o1 - o0, "bytes": b1 - b0, "groups": g1 - g0, "s": round(t, 2)}), flush=True)

if __name__ == "__main__":
    main()
