#!/bin/bash
# Round 4: the sort without the tie flags' sync (speculative, default) against KHST_SPEC=0, 100M,
# alternating on one box, roots checked
export TMPDIR=/tmp
tag=${1:-r4ac}
ROOT=577f095224664dc395ca23578afe7bd0c82dbeb5a863285af99e8271a81b9cad
step() { local name=$1; shift; "$@"; local rc=$?; echo "${name}_RC=$rc" >&2; [ $rc -eq 0 ] || exit $rc; }
for v in 1 0 1b 0b 1c 0c; do
  step BENCH_$v env KHST_SPEC=${v:0:1} timeout -k 10 300 python bench.py --no-cpu --no-host-path > gpurun_out/bench_${tag}_$v.json 2> gpurun_out/bench_${tag}_$v.err
  grep -q $ROOT gpurun_out/bench_${tag}_$v.json || { echo "ROOT MISMATCH $v"; exit 3; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], round(d['ms_per_step'],2), {k: round(x,2) for k,x in d['stage_ms'].items()})" gpurun_out/bench_${tag}_$v.json $v
done
