"""Cuts a rocprofv3 kernel trace of scripts/block_commit_prof.py into its commits (idle gaps
> --gap ms) and reports, for the last --blocks windows: launches, summed kernel time, the
window's span (first start to last end) and the largest kernels.  Measurement only.

  python scripts/block_trace.py gpurun_out/bc [--blocks 3] [--gap 30]
"""
import argparse
import collections
import csv
import glob
import json


def main():
    p = argparse.ArgumentParser()
    p.add_argument("dir")
    p.add_argument("--blocks", type=int, default=3)
    p.add_argument("--gap", type=float, default=30.0)
    p.add_argument("--timeline", default=None, help="write the last window's launches to this JSON file")
    a = p.parse_args()
    rows = []
    for f in glob.glob(f"{a.dir}/**/*kernel_trace.csv", recursive=True):
        rows += list(csv.DictReader(open(f)))
    ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0],
                 r.get("Queue_Id", r.get("Stream_Id", "0"))) for r in rows)
    wins, cur = [], []
    for e in ev:
        if cur and e[0] - max(x[1] for x in cur[-8:]) > a.gap * 1e6:
            wins.append(cur)
            cur = []
        cur.append(e)
    if cur:
        wins.append(cur)
    out = []
    for w in wins[-a.blocks:]:
        busy = sum(e[1] - e[0] for e in w) / 1e6
        span = (max(e[1] for e in w) - w[0][0]) / 1e6
        # the time any kernel runs (union of intervals): busy above it means concurrent queues
        union, cs, ce = 0, None, None
        for e in sorted(w):
            if ce is None or e[0] > ce:
                if ce is not None:
                    union += ce - cs
                cs, ce = e[0], e[1]
            else:
                ce = max(ce, e[1])
        union = (union + (ce - cs if ce is not None else 0)) / 1e6
        queues = collections.Counter(e[3] for e in w)
        per = collections.defaultdict(lambda: [0, 0.0])
        for e in w:
            k = e[2].replace("void ", "").replace("khst::", "").split("<")[0]
            per[k][0] += 1
            per[k][1] += (e[1] - e[0]) / 1e6
        top = sorted(per.items(), key=lambda kv: -kv[1][1])[:12]
        out.append({"launches": len(w), "kernel_ms": round(busy, 3), "span_ms": round(span, 3),
                    "idle_in_span_ms": round(span - union, 3), "any_kernel_running_ms": round(union, 3),
                    "launches_per_queue": dict(queues),
                    "top": {k: {"n": v[0], "ms": round(v[1], 3)} for k, v in top}})
    if a.timeline and wins:  # the last window launch by launch: start offset, duration, gap before
        w = wins[-1]
        t0, prev = w[0][0], w[0][0]
        tl = []
        for e in w:
            k = e[2].replace("void ", "").replace("khst::", "").split("<")[0][:40]
            tl.append([k, round((e[0] - t0) / 1e3, 1), round((e[1] - e[0]) / 1e3, 1), round((e[0] - prev) / 1e3, 1),
                       e[3]])
            prev = max(prev, e[1])
        with open(a.timeline, "w") as f:
            json.dump({"columns": ["kernel", "start_us", "dur_us", "gap_before_us", "queue"], "launches": tl}, f)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
