#!/bin/bash
# kernel timeline of the 100M step (both streams): rocprofv3 kernel trace of a short bench run
export TMPDIR=/tmp
tag=${1:-st}
step() { local name=$1; shift; "$@"; local rc=$?; echo "${name}_RC=$rc" >&2; [ $rc -eq 0 ] || exit $rc; }
step ST timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/st_$tag -o st -- python3 bench.py --steps 2 --warmup 1 --no-cpu > gpurun_out/st_$tag.log 2>&1
python3 scripts/step_timeline.py gpurun_out/st_$tag > gpurun_out/step_timeline_$tag.json && cut -c1-300 gpurun_out/step_timeline_$tag.json
