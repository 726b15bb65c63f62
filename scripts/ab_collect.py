"""Collect scripts/gpu_ab_fetch.sh runs (gpurun_out/ab_<tag>_<label>_<rep>.json) into one
profiles/ record (measurement only):  python scripts/ab_collect.py TAG OUT.json "what" [label=desc ...]"""
import glob
import json
import re
import sys


def main():
    tag, out, what = sys.argv[1], sys.argv[2], sys.argv[3]
    desc = dict(a.split("=", 1) for a in sys.argv[4:])
    runs = {}
    for f in sorted(glob.glob(f"gpurun_out/ab_{tag}_*.json")):
        m = re.match(rf"gpurun_out/ab_{tag}_(.+)_(\d+)\.json$", f)
        d = json.loads(open(f).read().strip().splitlines()[-1])
        runs.setdefault(m.group(1), []).append({"rep": int(m.group(2)), "ms_per_step": round(d["ms_per_step"], 3),
                                                "state_root": d["state_root"],
                                                "stage_ms": {k: round(v, 3) for k, v in d["stage_ms"].items()}})
    json.dump({"what": what, "builds": desc, "runs": runs}, open(out, "w"), indent=1)
    for k, v in runs.items():
        print(k, [r["ms_per_step"] for r in v])


if __name__ == "__main__":
    main()
