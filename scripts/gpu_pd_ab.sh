#!/bin/bash
# A/B of where the early leaves' parent depths are scattered (KHST_PD), with the parity
# tests of the plain-root path under each folded mode first (measurement only)
export TMPDIR=/tmp
tag=${1:-pd}
for mode in ${PD_MODES:-ansv chain}; do
  KHST_PD=$mode timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_${tag}_$mode.log 2>&1; rc=$?; tail -1 gpurun_out/pytest_${tag}_$mode.log; [ $rc -eq 0 ] || exit $rc
done
bash scripts/gpu_ab_lib.sh $tag "sep:KHST_PD=sep" "ansv:KHST_PD=ansv" "chain:KHST_PD=chain" "lcp:KHST_PD=lcp"
