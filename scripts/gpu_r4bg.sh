#!/bin/bash
# configs[2] block commits with k_branch_xl over larger levels (KHST_XL_LEVEL, default 8192)
export TMPDIR=/tmp
tag=${1:-r4bg}
step() { local name=$1; shift; "$@"; local rc=$?; echo "${name}_RC=$rc" >&2; [ $rc -eq 0 ] || exit $rc; }
for rep in 1 2; do
for v in def:X=1 x16k:KHST_XL_LEVEL=16384 x40k:KHST_XL_LEVEL=40000; do
  l=${v%%:*}; e=${v#*:}
  step CFG2_$l env $e timeout -k 10 400 python scripts/bench_configs.py --cfg 3 --no-cpu > gpurun_out/${tag}_cfg2_${l}_$rep.jsonl 2> gpurun_out/${tag}_cfg2_${l}_$rep.err
  python -c "import json;d=json.loads(open('gpurun_out/${tag}_cfg2_${l}_$rep.jsonl').readline());print('$l', round(d['block_ms_median'],3), [round(x,3) for x in d['block_ms_all']])"
done
done
echo done
