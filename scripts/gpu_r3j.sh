#!/bin/bash
# round 3: leaf link records (no copy pass after the join) -- parity, A/B against the
# copy pass (KHST_LEAF_MOVE=1), then the storage line's HIP API trace
export TMPDIR=/tmp
tag=${1:-r3j}
step() { local name=$1; shift; "$@"; local rc=$?; echo "${name}_RC=$rc" >&2; [ $rc -eq 0 ] || exit $rc; }
step PYTEST timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_lists.py tests/test_gpu_configs.py tests/test_gpu_sharded_cabi.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_$tag.log 2>&1
tail -1 gpurun_out/pytest_$tag.log
step AB bash scripts/gpu_ab_lib.sh $tag "links:X=1" "move:KHST_LEAF_MOVE=1"
step ST timeout -k 10 300 rocprofv3 --kernel-trace --hip-trace --stats --output-format csv -d gpurun_out/st_$tag -o st -- python3 bench.py --workload storage --steps 3 --warmup 1 --no-cpu > gpurun_out/st_$tag.log 2>&1
