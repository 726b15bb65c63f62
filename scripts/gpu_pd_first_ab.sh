#!/bin/bash
# KHST_PD=first (the parent-depth scatter alone on the topology stream, then the leaves,
# the plain ANSV beside them) against the default (scatter folded into the ANSV), 100M
export TMPDIR=/tmp
tag=${1:-pf}
KHST_PD=first timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_${tag}_first.log 2>&1; rc=$?; tail -1 gpurun_out/pytest_${tag}_first.log; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_ab_lib.sh $tag "def:KHST_PD=ansv" "first:KHST_PD=first"
