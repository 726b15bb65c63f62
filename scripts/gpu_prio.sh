#!/bin/bash
# A/B of the stream priorities (KHST_LEAF_PRIO) on the 100M bench, no CPU legs.
export TMPDIR=/tmp
for p in lo hi lo hi; do
  KHST_LEAF_PRIO=$p timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu > gpurun_out/prio_$p.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('gpurun_out/prio_$p.json'));print('$p', round(d['ms_per_step'],2), {k: round(v,2) for k,v in d['stage_ms'].items()})"
done
