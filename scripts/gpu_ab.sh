#!/bin/bash
# A/B of an env switch on the 100M bench: bash scripts/gpu_ab.sh VAR v1 v2 ...
export TMPDIR=/tmp
var=$1; shift
for rep in 1 2; do
for v in "$@"; do
  env $var=$v timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu > gpurun_out/ab_${var}_$v.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('gpurun_out/ab_${var}_$v.json'));print('$var=$v', round(d['ms_per_step'],2), d['state_root'][:12], {k: round(v,2) for k,v in d['stage_ms'].items()})"
done
done
