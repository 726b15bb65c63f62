#!/bin/bash
# Round 4: tile-local topology (k_topo_tile).  Parity tests, then 100M A/B against the
# whole-array ANSV / chain (KHST_TOPO_TILE=0), every line's root checked against the pinned
# 100M root; then a kernel trace of the default and the world-8 shard-build simulation.
export TMPDIR=/tmp
tag=${1:-r4k}
ROOT=577f095224664dc395ca23578afe7bd0c82dbeb5a863285af99e8271a81b9cad
step() { local name=$1; shift; "$@"; local rc=$?; echo "${name}_RC=$rc" >&2; [ $rc -eq 0 ] || exit $rc; }
step PYTEST timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_lists.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_${tag}.log 2>&1
tail -1 gpurun_out/pytest_${tag}.log
for v in old new old2 new2; do
  case $v in old*) envs="KHST_TOPO_TILE=0" ;; new*) envs="KHST_TOPO_TILE=1" ;; esac
  step BENCH_$v env $envs timeout -k 10 300 python bench.py --no-cpu --no-host-path > gpurun_out/bench_${tag}_$v.json 2> gpurun_out/bench_${tag}_$v.err
  grep -q $ROOT gpurun_out/bench_${tag}_$v.json || { echo "ROOT MISMATCH $v"; exit 3; }
  cut -c1-200 gpurun_out/bench_${tag}_$v.json
done
step PROF timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$tag -o run -- python3 bench.py --no-cpu --no-host-path --steps 5 --warmup 2 > gpurun_out/prof_${tag}.json 2> gpurun_out/prof_${tag}.err
step SIM timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/sim_$tag -o sim -- python3 scripts/shard_rank_sim.py --world 8 > gpurun_out/sim_$tag.json 2> gpurun_out/sim_$tag.err
cut -c1-600 gpurun_out/sim_$tag.json
