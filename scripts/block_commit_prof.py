"""configs[2] block commits under a kernel trace (measurement only): the 50M-account
resident state of tests/blocks.py, `--warmup` blocks, then `--blocks` blocks whose inputs are
made first, each commit separated by an idle gap so scripts/block_trace.py can cut the
trace into blocks.  Run under rocprofv3 --kernel-trace:

  rocprofv3 --kernel-trace --stats -d gpurun_out/bc -o bc -- python scripts/block_commit_prof.py
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--resident", type=int, default=50_000_000)
    p.add_argument("--warmup", type=int, default=2)
    p.add_argument("--blocks", type=int, default=3)
    p.add_argument("--gap-ms", type=float, default=60.0)
    a = p.parse_args()
    import torch
    from khipu_amd.device import Ctx
    from tests.blocks import BlockWorkload
    ctx = Ctx(0)
    nb = a.warmup + a.blocks
    w = BlockWorkload(ctx, a.resident, nb)
    for b in range(a.warmup):
        w.block(b)
    ops = [w.prepare(a.warmup + i) for i in range(a.blocks)]
    torch.cuda.synchronize()
    wall = []
    for o in ops:
        time.sleep(a.gap_ms / 1e3)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        w.commit_prepared(o)
        torch.cuda.synchronize()
        wall.append((time.perf_counter() - t0) * 1e3)
    time.sleep(a.gap_ms / 1e3)
    print(json.dumps({"resident": a.resident, "block_wall_ms": [round(x, 3) for x in wall]}), flush=True)


if __name__ == "__main__":
    main()
