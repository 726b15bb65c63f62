#!/bin/bash
# A/B of library builds on configs[2] block commits at 50M (measurement only):
#   bash scripts/gpu_bc_ab.sh TAG label=path ...   (path "" = the default libkhst.so)
# REPS (default 2) rounds over the builds; STEPS blocks timed per run.
export TMPDIR=/tmp
tag=$1; shift
for rep in $(seq 1 ${REPS:-2}); do
for spec in "$@"; do
  label=${spec%%=*}; lib=${spec#*=}
  KHST_LIB_AB=$lib timeout -k 10 300 python scripts/bench_configs.py --cfg 3 --steps ${STEPS:-10} --warmup 2 --no-cpu \
    > gpurun_out/bcab_${tag}_${label}_$rep.json 2>gpurun_out/bcab_${tag}_${label}_$rep.err || { tail -5 gpurun_out/bcab_${tag}_${label}_$rep.err; exit 1; }
  python -c "
import json
d=[json.loads(x) for x in open('gpurun_out/bcab_${tag}_${label}_$rep.json') if x.startswith('{')][-1]
print('$label', round(d['block_ms_median'],3), sorted(round(x,3) for x in d['block_ms_all']), d['state_root_after'][:12])"
done
done
