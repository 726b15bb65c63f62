#!/bin/bash
# Per-kernel averages of configs[2] block commits at 50M under a kernel trace, per library build
# (measurement only):  bash scripts/gpu_bc_kstats_ab.sh TAG label=path ...  (path "" = default)
export TMPDIR=/tmp
tag=$1; shift
for spec in "$@"; do
  label=${spec%%=*}; lib=${spec#*=}
  KHST_LIB_AB=$lib timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/bck_${tag}_$label -o bc \
    -- python3 scripts/block_commit_prof.py --blocks 6 > gpurun_out/bck_${tag}_$label.log 2>&1 || { tail -5 gpurun_out/bck_${tag}_$label.log; exit 1; }
  python3 - "$label" gpurun_out/bck_${tag}_$label <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[2] + "/**/*kernel_stats.csv", recursive=True)[0]
rows = {r["Name"].split("(")[0]: r for r in csv.DictReader(open(f))}
want = ["k_f_gather", "k_f_descend", "k_f_elem_flags", "k_map_delete", "k_f_branch_recs"]
print(sys.argv[1], {k: round(float(rows[k]["AverageNs"]) / 1e3, 1) for k in want if k in rows})
PY
done
