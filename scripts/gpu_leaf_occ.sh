#!/bin/bash
# A/B of the leaf kernel's occupancy cap (KHST_LEAF_DYN_LDS bytes of extra LDS per block).
export TMPDIR=/tmp
for d in 0 30000 43000 70000 0; do
  KHST_LEAF_DYN_LDS=$d timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu > gpurun_out/occ_$d.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('gpurun_out/occ_$d.json'));print('$d', round(d['ms_per_step'],2), {k: round(v,2) for k,v in d['stage_ms'].items()})"
done
