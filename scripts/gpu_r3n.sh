#!/bin/bash
# round 3: the leaf copy pass split at one below the busiest branch level, its second part
# beside the deeper levels -- parity, then A/B against one pass (KHST_MOVE_SPLIT=0) at 100M
export TMPDIR=/tmp
tag=${1:-r3n}
step() { local name=$1; shift; "$@"; local rc=$?; echo "${name}_RC=$rc" >&2; [ $rc -eq 0 ] || exit $rc; }
step PYTEST timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_$tag.log 2>&1
tail -1 gpurun_out/pytest_$tag.log
step AB bash scripts/gpu_ab_lib.sh $tag "split:KHST_MOVE_SPLIT=1" "one:X=1"
