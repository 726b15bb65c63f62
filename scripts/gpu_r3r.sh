#!/bin/bash
# round 3: branch levels in one-wave blocks (KHST_BRANCH_BS=64: 18 waves per CU instead of
# 16) -- parity under the switch, then A/B at 100M
export TMPDIR=/tmp
tag=${1:-r3r}
step() { local name=$1; shift; "$@"; local rc=$?; echo "${name}_RC=$rc" >&2; [ $rc -eq 0 ] || exit $rc; }
step PYTEST env KHST_BRANCH_BS=64 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_$tag.log 2>&1
tail -1 gpurun_out/pytest_$tag.log
step AB bash scripts/gpu_ab_lib.sh $tag "bs64:KHST_BRANCH_BS=64" "bs256:X=1"
