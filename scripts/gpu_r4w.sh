#!/bin/bash
# configs[2] block commit at 50M: tile-local topology (default) vs the whole-array ANSV / chain
# (KHST_TOPO_TILE=0) in the element builds, alternating on one box
export TMPDIR=/tmp
tag=${1:-r4w}
step() { local name=$1; shift; "$@"; local rc=$?; echo "${name}_RC=$rc" >&2; [ $rc -eq 0 ] || exit $rc; }
for v in 1 0 1b 0b; do
  step CFG3_$v env KHST_TOPO_TILE=${v:0:1} timeout -k 10 300 python scripts/bench_configs.py --cfg 3 --no-cpu > gpurun_out/cfg3_${tag}_$v.json 2> gpurun_out/cfg3_${tag}_$v.err
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], round(d['block_ms_median'],3), [round(x,3) for x in d['block_ms_all']])" gpurun_out/cfg3_${tag}_$v.json $v
done
