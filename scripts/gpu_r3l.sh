#!/bin/bash
# round 3: occupancy A/B -- leaf kernel at 7 waves/SIMD (72 VGPRs, working tree) vs HEAD
# (6 waves), and key hashing forced to 8 waves (64 VGPRs + spills)
export TMPDIR=/tmp
tag=${1:-r3l}
step() { local name=$1; shift; "$@"; local rc=$?; echo "${name}_RC=$rc" >&2; [ $rc -eq 0 ] || exit $rc; }
step PYTEST timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_$tag.log 2>&1
tail -1 gpurun_out/pytest_$tag.log
step AB bash scripts/gpu_ab_lib.sh $tag "w7:X=1" "head:KHST_LIB_AB=khipu_amd/libkhst_base.so" "k8:KHST_LIB_AB=khipu_amd/libkhst_k8.so"
