#!/bin/bash
# round 3: fused theta (180 VALU per round) -- smoke parity, then A/B against HEAD's library
export TMPDIR=/tmp
tag=${1:-r3d}
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_$tag.log 2>&1 || { tail -40 gpurun_out/pytest_$tag.log; exit 1; }
tail -1 gpurun_out/pytest_$tag.log
bash scripts/gpu_ab_lib.sh $tag "new:X=1" "base:KHST_LIB_AB=khipu_amd/libkhst_base.so" || exit 1
