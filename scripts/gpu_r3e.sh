#!/bin/bash
# round 3: leaves hashed in sorted order (KHST_LEAF=sorted) -- parity under the switch, A/B
export TMPDIR=/tmp
tag=${1:-r3e}
KHST_LEAF=sorted timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_$tag.log 2>&1 || { tail -40 gpurun_out/pytest_$tag.log; exit 1; }
tail -1 gpurun_out/pytest_$tag.log
bash scripts/gpu_ab_lib.sh $tag "input:X=1" "sorted:KHST_LEAF=sorted" || exit 1
