"""Host-side view of configs[2] block commits (measurement only): a rocprofv3 --hip-trace
--kernel-trace run of scripts/block_commit_prof.py, cut into blocks at the idle gaps, then per
block and host thread: time inside HIP calls by function, the host time between a
hipStreamSynchronize returning and the thread's next HIP call, and for every kernel the delay
from its launch call returning to the kernel starting on the GPU.

  python scripts/api_trace.py gpurun_out/bch_r6d > profiles/<tag>_block_commit_host_api_50m.json
"""
import collections
import csv
import glob
import json
import sys


def rows(d, pat):
    out = []
    for f in glob.glob(f"{d}/**/{pat}", recursive=True):
        out += list(csv.DictReader(open(f)))
    return out


def main():
    d = sys.argv[1]
    gap_ns = 20e6
    api = rows(d, "*hip_api_trace.csv")
    ker = rows(d, "*kernel_trace.csv")
    ks = sorted(({"name": r["Kernel_Name"].split("(")[0].replace("void ", ""), "corr": r["Correlation_Id"],
                  "s": int(r["Start_Timestamp"]), "e": int(r["End_Timestamp"])} for r in ker), key=lambda k: k["s"])
    # blocks: kernels separated by idle gaps
    blocks, cur = [], []
    for k in ks:
        if cur and k["s"] - max(x["e"] for x in cur) > gap_ns:
            blocks.append(cur)
            cur = []
        cur.append(k)
    blocks.append(cur)
    blocks = [b for b in blocks if len(b) > 50][-3:]  # the timed blocks
    calls = sorted(({"fn": r["Function"], "tid": r["Thread_Id"], "corr": r["Correlation_Id"], "s": int(r["Start_Timestamp"]),
                     "e": int(r["End_Timestamp"])} for r in api), key=lambda c: c["s"])
    by_corr = {c["corr"]: c for c in calls}
    res = []
    for b in blocks:
        t0, t1 = b[0]["s"] - 200_000, max(k["e"] for k in b)
        cs = [c for c in calls if t0 <= c["s"] <= t1]
        per_thread = collections.defaultdict(list)
        for c in cs:
            per_thread[c["tid"]].append(c)
        threads = {}
        for tid, lst in per_thread.items():
            fn_us = collections.Counter()
            fn_n = collections.Counter()
            after_sync = []
            for i, c in enumerate(lst):
                fn_us[c["fn"]] += (c["e"] - c["s"]) / 1e3
                fn_n[c["fn"]] += 1
                if c["fn"] == "hipStreamSynchronize" and i + 1 < len(lst):
                    after_sync.append(round((lst[i + 1]["s"] - c["e"]) / 1e3, 1))
            span = (lst[-1]["e"] - lst[0]["s"]) / 1e3
            threads[tid] = {"calls": len(lst), "span_us": round(span, 1),
                            "in_hip_us": round(sum(fn_us.values()), 1),
                            "by_function_us": {k: [fn_n[k], round(v, 1)] for k, v in fn_us.most_common(12)},
                            "host_us_after_each_sync": after_sync}
        lat = []
        for k in b:
            c = by_corr.get(k["corr"])
            if c:
                lat.append((k["s"] - c["e"]) / 1e3)
        lat.sort()
        res.append({"kernels": len(b), "gpu_span_us": round((t1 - b[0]["s"]) / 1e3, 1), "threads": threads,
                    "launch_return_to_kernel_start_us": {"median": round(lat[len(lat) // 2], 1) if lat else None,
                                                         "p90": round(lat[int(len(lat) * 0.9)], 1) if lat else None}})
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
