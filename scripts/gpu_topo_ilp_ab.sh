#!/bin/bash
# 100M A/B: k_chain / k_branch_topo walking 4 boundaries per thread in lockstep
# (KHST_TOPO_ILP=1) at topology grid caps of 1, 2 and 4 blocks per CU, against the default;
# every line's state root is checked against the pinned 100M root
export TMPDIR=/tmp
tag=${1:-til}
ROOT=577f095224664dc395ca23578afe7bd0c82dbeb5a863285af99e8271a81b9cad
step() { local name=$1; shift; "$@"; local rc=$?; echo "${name}_RC=$rc" >&2; [ $rc -eq 0 ] || exit $rc; }
for v in def ilp4 ilp2 ilp1 def2 ilp2b; do
  case $v in
    def*) envs="KHST_TOPO_ILP=0" ;;
    ilp4) envs="KHST_TOPO_ILP=1 KHST_TOPO_BPC=4" ;;
    ilp2*) envs="KHST_TOPO_ILP=1 KHST_TOPO_BPC=2" ;;
    ilp1) envs="KHST_TOPO_ILP=1 KHST_TOPO_BPC=1" ;;
  esac
  step BENCH_$v env $envs timeout -k 10 300 python bench.py --no-cpu > gpurun_out/bench_${tag}_$v.json 2> gpurun_out/bench_${tag}_$v.err
  grep -q $ROOT gpurun_out/bench_${tag}_$v.json || { echo "ROOT MISMATCH $v"; exit 3; }
  cut -c1-200 gpurun_out/bench_${tag}_$v.json
done
