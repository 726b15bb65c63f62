"""Summarise the rocprofv3 PMC passes of scripts/gpu_pmc.sh per kernel.

usage: python scripts/pmc_summary.py <tag> [builds] [--json out.json]

Counters are summed over every dispatch of a kernel and divided by the number of
builds the profiled command ran (bench.py --steps 1 --warmup 1 -> 2 builds), so each
row is per build; `calls` is dispatches per build.  HBM bytes follow
MI355X_MICROARCH.md (HBM section): FETCH_SIZE counts 64 B per fabric read request and
reports half the bytes of a wide coalesced read, so the corrected read bytes are
2 x FETCH_SIZE(kB) x 1e3; WRITE_SIZE is taken as is.
"""
import collections
import csv
import glob
import json
import sys

out_json = sys.argv[sys.argv.index("--json") + 1] if "--json" in sys.argv else None
args = [a for a in sys.argv[1:] if not a.startswith("--") and a != out_json]
tag = args[0] if args else "pmc"
builds = int(args[1]) if len(args) > 1 else 2

def kname(full):
    """'void khst::k_scan_tiles<unsigned int>(...)' -> 'k_scan_tiles' (template instances merge)"""
    return full.split("(")[0].replace("void ", "").split("<")[0].replace("khst::", "").strip()


agg = collections.defaultdict(lambda: collections.defaultdict(float))
for f in sorted(glob.glob(f"gpurun_out/{tag}_p*/**/pmc_counter_collection.csv", recursive=True)):
    for r in csv.DictReader(open(f)):
        agg[kname(r["Kernel_Name"])][r["Counter_Name"]] += float(r["Counter_Value"])
dur = collections.defaultdict(float)
calls = collections.defaultdict(int)
vg = {}
for f in sorted(glob.glob(f"gpurun_out/{tag}_p1/**/pmc_kernel_trace.csv", recursive=True)):
    for r in csv.DictReader(open(f)):
        k = kname(r["Kernel_Name"])
        dur[k] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
        calls[k] += 1
        vg[k] = (r.get("VGPR_Count") or r.get("Arch_VGPR_Count"), r.get("LDS_Block_Size"))

rows = {}
print(f"{'kernel':26s} {'calls':>5s} {'ms':>8s} {'read MB':>9s} {'write MB':>9s} {'GB/s':>7s} {'VALU M':>8s} "
      f"{'valu%':>5s} {'wait%':>5s}  vgpr/lds")
for k in sorted(dur, key=lambda x: -dur[x]):
    a = agg[k]
    ms = dur[k] / builds
    rd = 2 * a["FETCH_SIZE"] * 1e3 / builds
    wr = a["WRITE_SIZE"] * 1e3 / builds
    cyc = max(a["SQ_WAVE_CYCLES"], 1)
    rows[k] = {"calls_per_build": calls[k] / builds, "ms_per_build": ms, "read_bytes": rd, "write_bytes": wr,
               "hbm_bytes": rd + wr, "valu_insts": a["SQ_INSTS_VALU"] / builds,
               "valu_active_frac": a["SQ_ACTIVE_INST_VALU"] / cyc, "wait_frac": a["SQ_WAIT_ANY"] / cyc}
    print(f"{k[:26]:26s} {calls[k] / builds:5.0f} {ms:8.3f} {rd / 1e6:9.1f} {wr / 1e6:9.1f} "
          f"{(rd + wr) / max(ms, 1e-9) / 1e6:7.0f} {a['SQ_INSTS_VALU'] / builds / 1e6:8.1f} "
          f"{100 * a['SQ_ACTIVE_INST_VALU'] / cyc:5.0f} {100 * a['SQ_WAIT_ANY'] / cyc:5.0f}  {vg.get(k)}")
if out_json:
    with open(out_json, "w") as f:
        json.dump({"tag": tag, "builds": builds, "hbm_correction": "read = 2 x FETCH_SIZE, write = WRITE_SIZE",
                   "kernels": rows}, f, indent=1)
