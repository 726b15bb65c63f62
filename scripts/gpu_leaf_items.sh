#!/bin/bash
export TMPDIR=/tmp
for d in 1 2 1 2; do
  KHST_LEAF_ITEMS=$d timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu > gpurun_out/items_$d.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('gpurun_out/items_$d.json'));print('$d', round(d['ms_per_step'],2), d['state_root'][:12], {k: round(v,2) for k,v in d['stage_ms'].items()})"
done
