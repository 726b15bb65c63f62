"""Per-kernel issue / wait breakdown from one rocprofv3 --pmc pass (scripts/gpu_r3p.sh).

SQ_* cycle counters count quad-cycles summed over waves (MI355X_MICROARCH.md, rocprofv3
section); GRBM_GUI_ACTIVE is summed over the 8 XCDs.  Per kernel: the fractions of wave
cycles parked on a wait (WAIT_ANY), stalled at issue (WAIT_INST_ANY) and issuing
(ACTIVE_INST_ANY / _VALU); the effective clock; and the SIMD VALU utilisation, the VALU
issue cycles summed over waves over (kernel time x 1,024 SIMDs x clock).

  python scripts/issue_summary.py gpurun_out/<dir> > profiles/<name>.json
"""
import collections
import csv
import glob
import json
import sys


def kname(full):
    return full.split("(")[0].replace("void ", "").split("<")[0].replace("khst::", "").strip()


def main():
    d = sys.argv[1]
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    for f in glob.glob(f"{d}/**/pmc_counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            agg[kname(r["Kernel_Name"])][r["Counter_Name"]] += float(r["Counter_Value"])
    dur = collections.defaultdict(float)
    for f in glob.glob(f"{d}/**/pmc_kernel_trace.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            dur[kname(r["Kernel_Name"])] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
    out = {}
    for k in sorted(dur, key=lambda x: -dur[x])[:12]:
        a = agg[k]
        cyc = max(a["SQ_WAVE_CYCLES"], 1.0)
        clk = a["GRBM_GUI_ACTIVE"] / 8 / dur[k] if dur[k] > 0 else 0.0
        waves = max(a["SQ_WAVES"], 1.0)
        out[k] = {"s": round(dur[k], 6), "clock_ghz": round(clk / 1e9, 3),
                  "wait_frac": round(a["SQ_WAIT_ANY"] / cyc, 3),
                  "issue_stall_frac": round(a["SQ_WAIT_INST_ANY"] / cyc, 3),
                  "active_frac": round(a["SQ_ACTIVE_INST_ANY"] / cyc, 3),
                  "active_valu_frac": round(a["SQ_ACTIVE_INST_VALU"] / cyc, 3),
                  "valu_per_unit": round(a["SQ_INSTS_VALU"] / waves, 1),
                  "salu_per_unit": round(a["SQ_INSTS_SALU"] / waves, 1),
                  "simd_valu_util": round(4 * a["SQ_ACTIVE_INST_VALU"] / (dur[k] * 1024 * clk), 3) if clk else None,
                  "wave_cycles_per_unit": round(4 * cyc / waves, 1)}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
