#!/bin/bash
# GPU parity suite, then an A/B of the leaf kernel on the 100M bench (measurement only)
export TMPDIR=/tmp
tag=${1:-leaf}
timeout -k 10 700 python -u -m pytest tests -x -v -m gpu --timeout 200 --timeout-method thread -o log_cli=false > gpurun_out/pytest_$tag.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_$tag.log; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_ab_lib.sh $tag "base:KHST_LIB_AB=khipu_amd/libkhst_base.so" "w5:KHST_LEAF_WPE=5" "w4:KHST_LEAF_WPE=4" "w6:KHST_LEAF_WPE=6"
