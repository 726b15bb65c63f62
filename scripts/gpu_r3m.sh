#!/bin/bash
# round 3: branch-stream prefill/padding trims and the 16-lane k_f_gather -- parity
# (parity, resident, configs), A/B against HEAD at 100M (and the parent-depth scatter in
# 4 / 8 target slices), block-commit trace at 50M
export TMPDIR=/tmp
tag=${1:-r3m}
step() { local name=$1; shift; "$@"; local rc=$?; echo "${name}_RC=$rc" >&2; [ $rc -eq 0 ] || exit $rc; }
step PYTEST timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_resident.py tests/test_gpu_configs.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_$tag.log 2>&1
tail -1 gpurun_out/pytest_$tag.log
step AB bash scripts/gpu_ab_lib.sh $tag "new:X=1" "head:KHST_LIB_AB=khipu_amd/libkhst_base.so" "c4:KHST_PD_CHUNKS=4" "c8:KHST_PD_CHUNKS=8"
step BC timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/bc_$tag -o bc -- python3 scripts/block_commit_prof.py > gpurun_out/bc_$tag.log 2>&1
python3 scripts/block_trace.py gpurun_out/bc_$tag > gpurun_out/bc_trace_$tag.json && head -30 gpurun_out/bc_trace_$tag.json
