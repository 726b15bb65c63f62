"""Per-dispatch FETCH_SIZE of one kernel family from scripts/gpu_ab_fetch.sh passes (the last
build's dispatches; rocprofv3 reports kB; read bytes = 2 x FETCH_SIZE on gfx950, as in scripts/pmc_summary.py):

  python scripts/fetch_by_dispatch.py TAG [kernel substring, default k_branch]"""
import csv
import glob
import sys

tag = sys.argv[1]
pat = sys.argv[2] if len(sys.argv) > 2 else "k_branch"
for d in sorted(glob.glob(f"gpurun_out/fetch_{tag}_*/")):
    rows = [r for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True) for r in csv.DictReader(open(f))]
    per = {}
    for r in rows:
        if pat in r["Kernel_Name"]:
            k = int(r["Dispatch_Id"])
            name = r["Kernel_Name"].split("(")[0].replace("void ", "")
            dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
            e = per.setdefault(k, [name, r["Grid_Size"], 0.0, dur])
            e[2] += float(r["Counter_Value"])
    ks = sorted(per)
    n_last = len(ks) // 2 if len(ks) % 2 == 0 else len(ks)  # warmup + timed build: the second half
    print(d)
    tot = 0.0
    for k in ks[-n_last:]:
        name, g, v, dur = per[k]
        gb = v * 1e3 * 2 / 1e9
        tot += gb
        print(f"  {name[:34]:34s} grid {g:>10s} fetch {gb:7.3f} GB  {dur:9.1f} us")
    print(f"  total {tot:.2f} GB")
