#!/bin/bash
# world-8 per-rank simulation: the topology kernels' grid cap and lockstep walk at the
# owner-shard size (12.5M records), alternated with the default on one box
export TMPDIR=/tmp
tag=${1:-tc}
step() { local name=$1; shift; "$@"; local rc=$?; echo "${name}_RC=$rc" >&2; [ $rc -eq 0 ] || exit $rc; }
for v in def bpc8 bpc0 ilp ilp8 def2 bpc8b bpc0b; do
  case $v in
    def*) envs="KHST_AB=none" ;;
    bpc8*) envs="KHST_TOPO_BPC=8" ;;
    bpc0*) envs="KHST_TOPO_BPC=0" ;;
    ilp) envs="KHST_TOPO_ILP=1" ;;
    ilp8) envs="KHST_TOPO_ILP=1 KHST_TOPO_BPC=8" ;;
  esac
  step SIM_$v env $envs timeout -k 10 300 python scripts/shard_rank_sim.py --world 8 > gpurun_out/sim_${tag}_$v.json 2> gpurun_out/sim_${tag}_$v.err
  python -c "import json;d=json.load(open('gpurun_out/sim_${tag}_$v.json'));print('$v', d['ms']['build'], {k: round(x,3) for k,x in d['build_stages_ms'].items()})"
done
