#!/bin/bash
# parity of the plain-root path with the scatter in k_lcp, then A/B of KHST_PD (measurement only)
export TMPDIR=/tmp
tag=${1:-pd2}
KHST_PD=lcp timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_${tag}.log 2>&1; rc=$?; tail -1 gpurun_out/pytest_${tag}.log; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_ab_lib.sh $tag "ansv:X=1" "lcp:KHST_PD=lcp" "lcp3:KHST_PD=lcp KHST_TOPO_BPC=3"
