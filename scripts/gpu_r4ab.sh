#!/bin/bash
# Round 4: the topology grid cap beside the leaf kernel re-measured with the tile topology
# (KHST_TOPO_BPC = blocks per CU of the beside-stream kernels), 100M, roots checked
export TMPDIR=/tmp
tag=${1:-r4ab}
ROOT=577f095224664dc395ca23578afe7bd0c82dbeb5a863285af99e8271a81b9cad
step() { local name=$1; shift; "$@"; local rc=$?; echo "${name}_RC=$rc" >&2; [ $rc -eq 0 ] || exit $rc; }
for v in 4 2 3 6 4b 2b 3b 6b; do
  step BENCH_$v env KHST_TOPO_BPC=${v:0:1} timeout -k 10 300 python bench.py --no-cpu --no-host-path > gpurun_out/bench_${tag}_$v.json 2> gpurun_out/bench_${tag}_$v.err
  grep -q $ROOT gpurun_out/bench_${tag}_$v.json || { echo "ROOT MISMATCH $v"; exit 3; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], round(d['ms_per_step'],2), {k: round(x,2) for k,x in d['stage_ms'].items()})" gpurun_out/bench_${tag}_$v.json $v
done
