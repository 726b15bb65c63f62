#!/bin/bash
# Round 4: sync tests (packed verify), the verify bench, the block-commit kernel trace at 50M
# (overlapped phases) with its per-queue timeline.
export TMPDIR=/tmp
TAG=${1:-r4g}
step() { local name=$1; shift; "$@"; local rc=$?; echo "${name}_RC=$rc" >&2; [ $rc -eq 0 ] || exit $rc; }
step PYTEST timeout -k 10 600 python -u -m pytest tests/test_gpu_sync.py -x -v -m gpu --timeout 300 --timeout-method thread -o log_cli=false > gpurun_out/pytest_$TAG.log 2>&1
tail -2 gpurun_out/pytest_$TAG.log
step VERIFY timeout -k 10 400 python bench.py --workload verify --steps 5 --warmup 2 > gpurun_out/bench_verify_$TAG.json 2> gpurun_out/bench_verify_$TAG.err
cut -c1-300 gpurun_out/bench_verify_$TAG.json
step BC timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/bc_$TAG -o bc -- python3 scripts/block_commit_prof.py > gpurun_out/bc_$TAG.log 2>&1
grep block_wall gpurun_out/bc_$TAG.log
python3 scripts/block_trace.py gpurun_out/bc_$TAG --timeline gpurun_out/bc_timeline_$TAG.json > gpurun_out/bc_trace_$TAG.json && head -12 gpurun_out/bc_trace_$TAG.json
