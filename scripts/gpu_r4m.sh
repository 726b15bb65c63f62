#!/bin/bash
# Round 4: schedules of the tile-local topology at 100M (KHST_TOPO_TILE=0 the whole-array
# ANSV / chain; 1 the scatter in k_topo_tile; 2 the scatter after it; 3 the scatter first, the
# leaves beside k_topo_tile), every root checked; then a kernel trace of mode 2
export TMPDIR=/tmp
tag=${1:-r4m}
ROOT=577f095224664dc395ca23578afe7bd0c82dbeb5a863285af99e8271a81b9cad
step() { local name=$1; shift; "$@"; local rc=$?; echo "${name}_RC=$rc" >&2; [ $rc -eq 0 ] || exit $rc; }
step PYTEST env KHST_TOPO_TILE=3 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_${tag}.log 2>&1
tail -1 gpurun_out/pytest_${tag}.log
for v in ${VARIANTS:-0 1 2 3 0b 3b 2b 1b}; do
  step BENCH_$v env KHST_TOPO_TILE=${v:0:1} timeout -k 10 300 python bench.py --no-cpu --no-host-path > gpurun_out/bench_${tag}_$v.json 2> gpurun_out/bench_${tag}_$v.err
  grep -q $ROOT gpurun_out/bench_${tag}_$v.json || { echo "ROOT MISMATCH $v"; exit 3; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], round(d['ms_per_step'],2), {k: round(x,2) for k,x in d['stage_ms'].items()})" gpurun_out/bench_${tag}_$v.json $v
done
step PROF env KHST_TOPO_TILE=2 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$tag -o run -- python3 bench.py --no-cpu --no-host-path --steps 5 --warmup 2 > gpurun_out/prof_${tag}.json 2> gpurun_out/prof_${tag}.err
