#!/bin/bash
# A/B of the small-level branch kernels at 50M block commits: default thresholds, every
# level up to 32,768 branches on the lane-spread kernel, and k_branch_fused everywhere
export TMPDIR=/tmp
tag=${1:-lv}
step() { local name=$1; shift; "$@"; local rc=$?; echo "${name}_RC=$rc" >&2; [ $rc -eq 0 ] || exit $rc; }
for v in default xl32k fused; do
  case $v in
    default) envs="" ;;
    xl32k) envs="KHST_XL_LEVEL=32768" ;;
    fused) envs="KHST_BRANCH_SMALL=0" ;;
  esac
  step BC_$v env $envs timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/lv_${tag}_$v -o lv -- python3 scripts/block_commit_prof.py > gpurun_out/lv_${tag}_$v.log 2>&1
  python3 scripts/block_trace.py gpurun_out/lv_${tag}_$v --timeline gpurun_out/lv_timeline_${tag}_$v.json > gpurun_out/lv_trace_${tag}_$v.json
  grep block_wall gpurun_out/lv_${tag}_$v.log
done
