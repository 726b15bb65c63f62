#!/bin/bash
# A/B of library builds on configs[3] (bench.py --workload storage, measurement only):
#   bash scripts/gpu_ab_storage.sh TAG label=path ...   (path "" = the default libkhst.so)
export TMPDIR=/tmp
tag=$1; shift
for rep in $(seq 1 ${REPS:-2}); do
for spec in "$@"; do
  label=${spec%%=*}; lib=${spec#*=}
  KHST_LIB_AB=$lib timeout -k 10 300 python bench.py --workload storage --steps 5 --warmup 1 --no-cpu > gpurun_out/abs_${tag}_${label}_$rep.json 2>/dev/null || exit 1
  python -c "import json;d=json.loads(open('gpurun_out/abs_${tag}_${label}_$rep.json').read().strip().splitlines()[-1]);print('$label', round(d['ms_per_step'],2), {k: round(v,2) for k,v in d['stage_ms_single_gpu_build'].items()})"
done
done
