"""Host side of the last block commit in a rocprofv3 --hip-trace (measurement only): every
HIP API call of the last window (cut like scripts/block_trace.py: idle gaps > --gap ms
between kernels), with its duration and the host time since the previous call ended.

  python scripts/api_trace.py gpurun_out/bc_api [--gap 30] [--top 40]
"""
import argparse
import csv
import glob
import json


def main():
    p = argparse.ArgumentParser()
    p.add_argument("dir")
    p.add_argument("--gap", type=float, default=30.0)
    p.add_argument("--top", type=int, default=40)
    a = p.parse_args()
    krows, arows = [], []
    for f in glob.glob(f"{a.dir}/**/*kernel_trace.csv", recursive=True):
        krows += list(csv.DictReader(open(f)))
    for f in glob.glob(f"{a.dir}/**/*hip_api_trace.csv", recursive=True):
        arows += list(csv.DictReader(open(f)))
    ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in krows)
    wins, cur = [], []
    for e in ev:
        if cur and e[0] - max(x[1] for x in cur[-8:]) > a.gap * 1e6:
            wins.append(cur)
            cur = []
        cur.append(e)
    if cur:
        wins.append(cur)
    w = wins[-1]
    t0, t1 = w[0][0] - 400_000, w[-1][1]  # (the call starts before its first kernel)
    calls = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Function"]) for r in arows
                   if t0 <= int(r["Start_Timestamp"]) <= t1)
    out, prev = [], None
    for s, e, fn in calls:
        out.append([fn, round((s - t0) / 1e3, 1), round((e - s) / 1e3, 1), round((s - prev) / 1e3, 1) if prev else 0.0])
        prev = e
    tot = {}
    for fn, _, d, _ in out:
        tot[fn] = tot.get(fn, 0.0) + d
    print(json.dumps({"calls": len(out), "api_us_by_function": dict(sorted(tot.items(), key=lambda kv: -kv[1])[:a.top]),
                      "host_gaps_over_10us": [x for x in out if x[3] > 10][:a.top],
                      "longest_calls": sorted(out, key=lambda x: -x[2])[:a.top]}, indent=1))


if __name__ == "__main__":
    main()
