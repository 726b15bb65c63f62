#!/bin/bash
# round 3: commit descent without hot-record atomics (touched flag read before it is
# exchanged, replacements counted per wave) -- resident/config parity, block-commit trace
# at 50M and the configs[2] line
export TMPDIR=/tmp
tag=${1:-r3s}
step() { local name=$1; shift; "$@"; local rc=$?; echo "${name}_RC=$rc" >&2; [ $rc -eq 0 ] || exit $rc; }
step PYTEST timeout -k 10 400 python -u -m pytest tests/test_gpu_resident.py tests/test_gpu_configs.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_$tag.log 2>&1
tail -1 gpurun_out/pytest_$tag.log
step BC timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/bc_$tag -o bc -- python3 scripts/block_commit_prof.py > gpurun_out/bc_$tag.log 2>&1
python3 scripts/block_trace.py gpurun_out/bc_$tag > gpurun_out/bc_trace_$tag.json && head -40 gpurun_out/bc_trace_$tag.json
step CFG2 timeout -k 10 400 python scripts/bench_configs.py --cfg 3 > gpurun_out/cfg2_$tag.jsonl 2> gpurun_out/cfg2_$tag.err
cut -c1-400 gpurun_out/cfg2_$tag.jsonl
