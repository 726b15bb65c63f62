#!/bin/bash
# GPU suite, then A/B of the topology grid cap in blocks per CU (measurement only)
export TMPDIR=/tmp
tag=${1:-cap}
timeout -k 10 700 python -u -m pytest tests -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/pytest_${tag}.log 2>&1; rc=$?; tail -1 gpurun_out/pytest_${tag}.log; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_ab_lib.sh $tag "base:KHST_LIB_AB=khipu_amd/libkhst_base.so" "bpc4:X=1" "bpc3:KHST_TOPO_BPC=3" "bpc5:KHST_TOPO_BPC=5" "bpc6:KHST_TOPO_BPC=6"
