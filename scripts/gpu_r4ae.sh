#!/bin/bash
# Round 4: kernel trace and launch timeline of configs[2] blocks at 50M after the early
# injection and the lazy commit tail
export TMPDIR=/tmp
TAG=${1:-r4ae}
step() { local name=$1; shift; "$@"; local rc=$?; echo "${name}_RC=$rc" >&2; [ $rc -eq 0 ] || exit $rc; }
step BC timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/bc_$TAG -o bc -- python3 scripts/block_commit_prof.py > gpurun_out/bc_$TAG.log 2>&1
python3 scripts/block_trace.py gpurun_out/bc_$TAG --timeline gpurun_out/bc_timeline_$TAG.json > gpurun_out/bc_trace_$TAG.json && head -12 gpurun_out/bc_trace_$TAG.json
