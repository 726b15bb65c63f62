#!/bin/bash
# A/B of library builds on the 100M bench plus one FETCH_SIZE pass per build (measurement only):
#   bash scripts/gpu_ab_fetch.sh TAG label=path ...   (path "" = the default libkhst.so)
# Summarise the passes with scripts/fetch_by_dispatch.py; NOFETCH=1 skips them.
export TMPDIR=/tmp
tag=$1; shift
specs=("$@")
for rep in $(seq 1 ${REPS:-2}); do
for spec in "${specs[@]}"; do
  label=${spec%%=*}; lib=${spec#*=}
  KHST_LIB_AB=$lib timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu --no-host-path > gpurun_out/ab_${tag}_${label}_$rep.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('gpurun_out/ab_${tag}_${label}_$rep.json'));print('$label', round(d['ms_per_step'],2), d['state_root'][:12], {k: round(v,2) for k,v in d['stage_ms'].items()})"
done
done
[ -n "$NOFETCH" ] && exit 0  # (NOFETCH=1: the timed runs only)
for spec in "${specs[@]}"; do
  label=${spec%%=*}; lib=${spec#*=}
  export KHST_LIB_AB=$lib
  timeout -s KILL 240 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d gpurun_out/fetch_${tag}_$label -o pmc \
    -- python3 bench.py --steps 1 --warmup 1 --no-cpu --no-host-path > gpurun_out/fetch_${tag}_$label.log 2>&1 || exit 1
  echo "FETCH_${label}_OK"
done
