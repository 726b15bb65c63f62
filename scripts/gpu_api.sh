#!/bin/bash
# host side of a block commit: rocprofv3 HIP API trace at 50M (scripts/api_trace.py)
export TMPDIR=/tmp
tag=${1:-api}
step() { local name=$1; shift; "$@"; local rc=$?; echo "${name}_RC=$rc" >&2; [ $rc -eq 0 ] || exit $rc; }
step API timeout -k 10 400 rocprofv3 --kernel-trace --hip-trace --output-format csv -d gpurun_out/bca_$tag -o bca -- python3 scripts/block_commit_prof.py > gpurun_out/bca_$tag.log 2>&1
python3 scripts/api_trace.py gpurun_out/bca_$tag > gpurun_out/api_$tag.json && head -80 gpurun_out/api_$tag.json
