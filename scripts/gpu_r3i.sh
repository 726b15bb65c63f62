#!/bin/bash
# round 3: where the storage line's wall time goes (HIP API + kernel trace, 3 steps)
export TMPDIR=/tmp
tag=${1:-r3i}
timeout -k 10 300 rocprofv3 --kernel-trace --hip-trace --stats --output-format csv -d gpurun_out/st_$tag -o st -- python3 bench.py --workload storage --steps 3 --warmup 1 --no-cpu > gpurun_out/st_$tag.log 2>&1
echo RC=$?
ls gpurun_out/st_$tag/*/ 2>/dev/null | head
