#!/bin/bash
# parity of the plain-root path, then A/B of the 16-byte stores (measurement only)
export TMPDIR=/tmp
tag=${1:-st4}
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_${tag}.log 2>&1; rc=$?; tail -1 gpurun_out/pytest_${tag}.log; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_ab_lib.sh $tag "base:KHST_LIB_AB=khipu_amd/libkhst_base.so" "nt:X=1"
bash scripts/gpu_ab_lib.sh ${tag}b "base:KHST_LIB_AB=khipu_amd/libkhst_base.so" "nt:X=1"
