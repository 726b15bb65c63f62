"""FETCH_SIZE / WRITE_SIZE per known byte for each access shape (scripts/fetch_calib.hip).

usage: python scripts/fetch_calib.py <rocprof dir of the FETCH_SIZE pass> <dir of the WRITE_SIZE pass>
                                     <stdout of fetch_calib> [--json out.json]"""
import collections
import csv
import glob
import json
import sys

rd_dir, wr_dir, known_txt = sys.argv[1:4]
out = sys.argv[sys.argv.index("--json") + 1] if "--json" in sys.argv else None
known = {}
for line in open(known_txt):
    p = line.split()
    if len(p) == 2 and p[1].isdigit():
        known[p[0]] = int(p[1])


def counters(d, name):
    c = collections.defaultdict(float)
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] == name:
                c[r["Kernel_Name"].split("(")[0].replace("void ", "").strip()] += float(r["Counter_Value"])
    return c


fs, ws = counters(rd_dir, "FETCH_SIZE"), counters(wr_dir, "WRITE_SIZE")
rows = {}
for k, b in known.items():
    if k.startswith("rd"):
        rows[k] = {"known_bytes": b, "FETCH_SIZE_bytes": fs[k] * 1e3, "ratio": fs[k] * 1e3 / b}
    else:
        rows[k] = {"known_bytes": b, "WRITE_SIZE_bytes": ws[k] * 1e3, "ratio": ws[k] * 1e3 / b}
    print(f"{k:10s} known {b / 1e9:8.3f} GB  counter/known = {rows[k]['ratio']:.3f}")
if out:
    with open(out, "w") as f:
        json.dump({"note": "counter bytes (kB x 1e3) / algorithmic bytes, per access shape; buffers 2 GiB (> L3)",
                   "shapes": rows}, f, indent=1)
