#!/bin/bash
# configs[2] block commits under a kernel trace, cut into blocks (measurement only):
#   bash scripts/gpu_block_trace.sh TAG
export TMPDIR=/tmp
TAG=${1:-bt}
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/bc_$TAG -o bc \
  -- python3 scripts/block_commit_prof.py > gpurun_out/bc_$TAG.log 2>&1 || { tail -20 gpurun_out/bc_$TAG.log; exit 1; }
tail -3 gpurun_out/bc_$TAG.log
python scripts/block_trace.py gpurun_out/bc_$TAG --timeline gpurun_out/bc_${TAG}_timeline.json > gpurun_out/bc_${TAG}_trace.json
head -c 600 gpurun_out/bc_${TAG}_trace.json
