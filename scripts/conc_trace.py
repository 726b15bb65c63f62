"""Summary of a kernel trace of scripts/concurrency_probe.py (measurement only): which HIP
streams ran on which hardware queues, and, over the probe's last phase (two threads
committing at once), how much of the time kernels of two streams overlapped.

  python scripts/conc_trace.py TRACE_DIR [--tail-ms MS]"""
import csv
import glob
import json
import sys
from collections import defaultdict


def main():
    d = sys.argv[1]
    tail_ms = float(sys.argv[sys.argv.index("--tail-ms") + 1]) if "--tail-ms" in sys.argv else 60.0
    rows = []
    for f in glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), int(r["Stream_Id"]), int(r["Queue_Id"]),
                             int(r["Thread_Id"]), r["Kernel_Name"].split("(")[0]))
    rows.sort()
    sq = defaultdict(lambda: [0, 0.0])
    for s, e, st, q, th, k in rows:
        sq[(st, q)][0] += 1
        sq[(st, q)][1] += (e - s) / 1e3
    t_end = rows[-1][1]
    tail = [r for r in rows if r[0] >= t_end - tail_ms * 1e6]
    # busy union over all kernels, and per stream
    def union(iv):
        iv = sorted(iv)
        tot, cs, ce = 0, iv[0][0], iv[0][1]
        for s, e in iv[1:]:
            if s > ce:
                tot += ce - cs
                cs, ce = s, e
            else:
                ce = max(ce, e)
        return tot + ce - cs
    by_stream = defaultdict(list)
    for s, e, st, q, th, k in tail:
        by_stream[st].append((s, e))
    span = tail[-1][1] - tail[0][0]
    out = {
        "streams_on_queues": {f"stream {st} -> queue {q}": {"kernels": n, "busy_ms": round(b, 2)} for (st, q), (n, b) in sorted(sq.items())},
        "tail_ms": round(span / 1e6, 2),
        "tail_busy_union_ms": round(union([(s, e) for s, e, *_ in tail]) / 1e6, 2),
        "tail_busy_per_stream_ms": {st: round(union(iv) / 1e6, 2) for st, iv in sorted(by_stream.items())},
        "tail_kernel_time_sum_ms": round(sum(e - s for s, e, *_ in tail) / 1e6, 2),
    }
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
