#!/bin/bash
# block commit at 50M: kernel trace + launch timeline, the configs[2] line, and the HIP API
# trace of the host side
export TMPDIR=/tmp
tag=${1:-bcapi}
step() { local name=$1; shift; "$@"; local rc=$?; echo "${name}_RC=$rc" >&2; [ $rc -eq 0 ] || exit $rc; }
step BC timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/bc_$tag -o bc -- python3 scripts/block_commit_prof.py > gpurun_out/bc_$tag.log 2>&1
grep block_wall gpurun_out/bc_$tag.log
python3 scripts/block_trace.py gpurun_out/bc_$tag --timeline gpurun_out/bc_timeline_$tag.json > gpurun_out/bc_trace_$tag.json && head -30 gpurun_out/bc_trace_$tag.json
step CFG2 timeout -k 10 400 python scripts/bench_configs.py --cfg 3 > gpurun_out/cfg2_$tag.jsonl 2> gpurun_out/cfg2_$tag.err
cut -c1-600 gpurun_out/cfg2_$tag.jsonl
step API timeout -k 10 400 rocprofv3 --kernel-trace --hip-trace --output-format csv -d gpurun_out/bca_$tag -o bca -- python3 scripts/block_commit_prof.py > gpurun_out/bca_$tag.log 2>&1
python3 scripts/api_trace.py gpurun_out/bca_$tag > gpurun_out/api_$tag.json && head -80 gpurun_out/api_$tag.json
