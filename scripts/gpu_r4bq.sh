#!/bin/bash
# Keccak straight-line (24 rounds unrolled) in the leaf kernel only, against HEAD (8 everywhere):
# the GPU suite, then the 100M step, 3 rounds alternated
export TMPDIR=/tmp
step() { local name=$1; shift; "$@"; local rc=$?; echo "${name}_RC=$rc" >&2; [ $rc -eq 0 ] || exit $rc; }
step PYTEST timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 200 --timeout-method thread -o log_cli=false > gpurun_out/r4bq_pytest.log 2>&1
grep -E "passed|failed" gpurun_out/r4bq_pytest.log | tail -1
step AB bash scripts/gpu_ab_lib.sh r4bq "base:KHST_LIB_AB=khipu_amd/libkhst_base.so" "leaf24:X=1"
step AB2 bash scripts/gpu_ab_lib.sh r4bq2 "leaf24:X=1" "base:KHST_LIB_AB=khipu_amd/libkhst_base.so"
echo done
