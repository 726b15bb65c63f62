"""Kernel timeline of a 100M step in a rocprofv3 --kernel-trace of bench.py (measurement
only): the kernels from one key-hashing launch to the next; every kernel with its start
offset, duration and queue (stream).

  python scripts/step_timeline.py gpurun_out/st [--gap 2] > timeline.json
"""
import argparse
import csv
import glob
import json


def main():
    p = argparse.ArgumentParser()
    p.add_argument("dir")
    p.add_argument("--gap", type=float, default=2.0)
    a = p.parse_args()
    rows = []
    for f in glob.glob(f"{a.dir}/**/*kernel_trace.csv", recursive=True):
        rows += list(csv.DictReader(open(f)))
    ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
                 r["Kernel_Name"].replace("void ", "").replace("khst::", "").split("(")[0].split("<")[0][:36],
                 r.get("Queue_Id", r.get("Stream_Id", "?"))) for r in rows)
    # a step starts at its key-hashing kernel: the last full step is the window between the
    # last two such starts that are followed by a whole step (the self-check build follows)
    starts = [i for i, e in enumerate(ev) if e[2].startswith("k_hash_keys")]
    if len(starts) >= 2:
        i0, i1 = starts[-2], starts[-1]
        w = ev[i0:i1]
    else:
        w = ev
    t0 = w[0][0]
    out = [[k, q, round((s - t0) / 1e6, 3), round((e - s) / 1e6, 3)] for s, e, k, q in w]
    print(json.dumps({"span_ms": round((max(x[1] for x in w) - t0) / 1e6, 3), "launches": len(w),
                      "columns": ["kernel", "queue", "start_ms", "dur_ms"], "kernels": out}))


if __name__ == "__main__":
    main()
