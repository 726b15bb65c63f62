#!/bin/bash
# GPU suite, then A/B of the leaf publish (measurement only)
export TMPDIR=/tmp
tag=${1:-link}
timeout -k 10 700 python -u -m pytest tests -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/pytest_${tag}.log 2>&1; rc=$?; tail -1 gpurun_out/pytest_${tag}.log; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_ab_lib.sh $tag "base:KHST_LIB_AB=khipu_amd/libkhst_base.so" "link:X=1" "move:KHST_PUBLISH=move"
