#!/bin/bash
# Keccak round loop unrolled 8 (default, 3 iterations) / 12 / 24 (straight-line): parity of
# the variants, then the 100M step A/B (builds khipu_amd/libkhst_u12.so / _u24.so, -DKECCAK_UNROLL)
export TMPDIR=/tmp
tag=${1:-r4bn}
step() { local name=$1; shift; "$@"; local rc=$?; echo "${name}_RC=$rc" >&2; [ $rc -eq 0 ] || exit $rc; }
step PYTEST env KHST_LIB_AB=khipu_amd/libkhst_u24.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 200 --timeout-method thread -o log_cli=false > gpurun_out/${tag}_pytest.log 2>&1
grep -E "passed|failed" gpurun_out/${tag}_pytest.log | tail -1
step AB bash scripts/gpu_ab_lib.sh $tag "u8:X=1" "u24:KHST_LIB_AB=khipu_amd/libkhst_u24.so" "u12:KHST_LIB_AB=khipu_amd/libkhst_u12.so"
echo done
