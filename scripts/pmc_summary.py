"""Summarise rocprofv3 PMC passes (scripts/gpu_pmc.sh output) per kernel, per call."""
import collections
import csv
import glob
import sys

tag = sys.argv[1] if len(sys.argv) > 1 else "pmc6"
agg = collections.defaultdict(lambda: collections.defaultdict(float))
for f in sorted(glob.glob(f"gpurun_out/{tag}_p*/pmc_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        agg[r["Kernel_Name"].split("(")[0]][r["Counter_Name"]] += float(r["Counter_Value"])
tr = list(csv.DictReader(open(f"gpurun_out/{tag}_p3/pmc_kernel_trace.csv")))
dur = collections.defaultdict(float)
calls = collections.defaultdict(int)
vg = {}
for r in tr:
    k = r["Kernel_Name"].split("(")[0]
    dur[k] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
    calls[k] += 1
    vg[k] = (r["VGPR_Count"], r["LDS_Block_Size"])
ncall = 2  # warmup + 1 step
print(f"{'kernel':24s} {'ms':>7s} {'FETCH MB':>9s} {'WRITE MB':>9s} {'VALU M':>8s} {'wait%':>5s}  vgpr/lds")
for k in sorted(dur, key=lambda x: -dur[x])[:int(sys.argv[2]) if len(sys.argv) > 2 else 20]:
    a = agg[k]
    print(f"{k[:24]:24s} {dur[k] / ncall:7.3f} {a['FETCH_SIZE'] / ncall / 1e3:9.1f} {a['WRITE_SIZE'] / ncall / 1e3:9.1f} "
          f"{a['SQ_INSTS_VALU'] / ncall / 1e6:8.1f} {100 * a['SQ_WAIT_ANY'] / max(a['SQ_WAVE_CYCLES'], 1):5.0f}  {vg[k]}")
