#!/bin/bash
# 100M schedule A/B after leaf positions: stream priorities (KHST_LEAF_PRIO=hi) and the
# topology kernels' grid cap (KHST_TOPO_BPC), alternated with the default on one box
export TMPDIR=/tmp
tag=${1:-sch}
step() { local name=$1; shift; "$@"; local rc=$?; echo "${name}_RC=$rc" >&2; [ $rc -eq 0 ] || exit $rc; }
for v in def prio bpc2 bpc8 def2; do
  case $v in
    def*) envs="KHST_LEAF_POS=1" ;;
    prio) envs="KHST_LEAF_PRIO=hi" ;;
    bpc2) envs="KHST_TOPO_BPC=2" ;;
    bpc8) envs="KHST_TOPO_BPC=8" ;;
  esac
  step BENCH_$v env $envs timeout -k 10 300 python bench.py --no-cpu > gpurun_out/bench_${tag}_$v.json 2> gpurun_out/bench_${tag}_$v.err
  cut -c1-200 gpurun_out/bench_${tag}_$v.json
done
