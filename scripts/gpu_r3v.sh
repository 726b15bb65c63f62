#!/bin/bash
# round 3, session 2: HEAD check (smoke, whole GPU suite, default bench) and a block-commit
# kernel timeline at 50M (scripts/block_trace.py --timeline)
export TMPDIR=/tmp
tag=${1:-r3v}
step() { local name=$1; shift; "$@"; local rc=$?; echo "${name}_RC=$rc" >&2; [ $rc -eq 0 ] || exit $rc; }
step SMOKE timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/smoke_$tag.log 2>&1
step PYTEST timeout -k 10 700 python -u -m pytest tests -x -v -m gpu --timeout 200 --timeout-method thread -o log_cli=false > gpurun_out/pytest_$tag.log 2>&1
tail -2 gpurun_out/pytest_$tag.log
step BENCH timeout -k 10 600 python bench.py > gpurun_out/bench_$tag.json 2> gpurun_out/bench_$tag.err
cut -c1-600 gpurun_out/bench_$tag.json
step BC timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/bc_$tag -o bc -- python3 scripts/block_commit_prof.py > gpurun_out/bc_$tag.log 2>&1
python3 scripts/block_trace.py gpurun_out/bc_$tag --timeline gpurun_out/bc_timeline_$tag.json > gpurun_out/bc_trace_$tag.json && head -30 gpurun_out/bc_trace_$tag.json
