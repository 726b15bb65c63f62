"""Two threads committing configs[2]-shaped blocks to two resident (state, forest) pairs, against
one thread committing the same blocks to both pairs in turn (measurement; the test is
tests/test_gpu_threads.py::test_block_commits_on_two_host_handles_overlap).

  python scripts/concurrency_probe.py [host|device] [n] [blocks]

host: handles opened through the host entry points (private contexts), kh_block_commit_host;
device: each pair on a caller context of its own (Ctx), kh_block_commit with device inputs."""
import ctypes
import json
import os
import sys
import threading
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from khipu_amd import _lib  # noqa: E402
from khipu_amd._lib import check, lib  # noqa: E402
from khipu_amd.device import Ctx, block_commit_host  # noqa: E402
from tests.blocks import BlockWorkload  # noqa: E402
from tests.test_gpu_threads import _host_ops  # noqa: E402


def main():
    mode = sys.argv[1] if len(sys.argv) > 1 else "host"
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 1_000_000
    nb = int(sys.argv[3]) if len(sys.argv) > 3 else 12
    out = {"mode": mode, "n": n, "blocks": nb, "hw_queues": os.environ.get("GPU_MAX_HW_QUEUES")}
    if mode == "device":
        ws = [BlockWorkload(Ctx(0), n, nb, seed=21) for _ in range(4)]
        ops = [ws[0].prepare(b) for b in range(nb)]

        def run(w, t):
            t0 = time.perf_counter()
            for o in ops:
                w.commit_prepared(tuple(x.clone() if x is not None else None for x in o))
            t.append(time.perf_counter() - t0)
    else:
        ctx = Ctx(0)
        w = BlockWorkload(ctx, n, nb, seed=21)
        ops = [_host_ops(w.prepare(b)) for b in range(nb)]
        keys0 = w.keys.cpu().numpy()
        vals0 = w.vals[:int(w.voff[n])].cpu().numpy()
        voff0 = w.voff[:n + 1].cpu().numpy().astype(np.uint64)

        class H:
            def __init__(self, h):
                self.h, self.ctx, self.root = h, ctx, None
        ws = []
        for _ in range(4):
            sh, fh = ctypes.c_void_p(), ctypes.c_void_p()
            root = np.zeros(32, np.uint8)
            check(lib().kh_trie_open_host(keys0.ctypes.data, 32, vals0.ctypes.data, voff0.ctypes.data, n, 0,
                                          root.ctypes.data, ctypes.byref(sh)))
            check(lib().kh_forest_open(None, _lib.KH_HASH_KEYS, ctypes.byref(fh)))
            ws.append((H(sh), H(fh)))

        def run(p, t):
            t0 = time.perf_counter()
            for o in ops:
                block_commit_host(p[0], p[1], **o)
            t.append(time.perf_counter() - t0)
    torch.cuda.synchronize()
    t1 = []
    run(ws[0], t1)
    run(ws[1], t1)
    ts = [[], []]
    th = [threading.Thread(target=run, args=(ws[2 + k], ts[k])) for k in range(2)]
    t0 = time.perf_counter()
    for t in th:
        t.start()
    for t in th:
        t.join()
    tp = time.perf_counter() - t0
    out.update({"one_thread_ms_per_block": round(sum(t1) * 1e3 / (2 * nb), 3),
                "two_threads_ms_per_block": round(tp * 1e3 / (2 * nb), 3),
                "per_thread_ms_per_block": [round(t[0] * 1e3 / nb, 3) for t in ts],
                "throughput_x": round(sum(t1) / tp, 3)})
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
