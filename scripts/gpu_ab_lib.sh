#!/bin/bash
# A/B of builds and env switches on the 100M bench (measurement only):
#   bash scripts/gpu_ab_lib.sh TAG "label:ENV=V ..." ...   (ENV may be KHST_LIB_AB=path)
export TMPDIR=/tmp
tag=$1; shift
for rep in $(seq 1 ${REPS:-2}); do
for spec in "$@"; do
  label=${spec%%:*}; envs=${spec#*:}
  env $envs timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu --no-host-path > gpurun_out/ab_${tag}_${label}_$rep.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('gpurun_out/ab_${tag}_${label}_$rep.json'));print('$label', round(d['ms_per_step'],2), d['state_root'][:12], {k: round(v,2) for k,v in d['stage_ms'].items()})"
done
done
