#!/bin/bash
# A/B (measurement only): radix tile size builds, stream priority / CU-mask schedules
export TMPDIR=/tmp
tag=${1:-sched}
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 120 --timeout-method thread -k "full_size or random or genesis" > gpurun_out/pytest_${tag}_rs16.log 2>&1; rc=$?
bash scripts/gpu_ab_lib.sh $tag "base:X=1" "rs16:KHST_LIB_AB=khipu_amd/libkhst_rs16.so" "rs32:KHST_LIB_AB=khipu_amd/libkhst_rs32.so" "eq:KHST_LEAF_PRIO=eq" "cu3:KHST_TOPO_CUQ=3" "cu2:KHST_TOPO_CUQ=2"
