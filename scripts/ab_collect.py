"""Collects the per-run JSON lines of scripts/gpu_ab_lib.sh into one profile:

  python scripts/ab_collect.py TAG "what the A/B compared" > profiles/<name>.json
"""
import glob
import json
import os
import sys


def main():
    tag, what = sys.argv[1], sys.argv[2]
    runs = []
    for p in sorted(glob.glob(f"gpurun_out/ab_{tag}_*.json")):
        d = json.load(open(p))
        runs.append({"run": os.path.basename(p), "ms_per_step": round(d["ms_per_step"], 3),
                     "state_root": d["state_root"],
                     "stage_ms": {k: round(v, 3) for k, v in d["stage_ms"].items()}})
    by = {}
    for r in runs:
        by.setdefault(r["run"][len(f"ab_{tag}_"):].rsplit("_", 1)[0], []).append(r["ms_per_step"])
    print(json.dumps({"what": what, "runs": runs,
                      "mean_ms_per_step": {k: round(sum(v) / len(v), 3) for k, v in by.items()}}, indent=1))


if __name__ == "__main__":
    main()
