#!/bin/bash
# round 3: kernel summaries of the current 100M step, in the step and serialized
export TMPDIR=/tmp
TAG=${1:-r3o}
step() { local name=$1; shift; "$@"; local rc=$?; echo "${name}_RC=$rc" >&2; [ $rc -eq 0 ] || exit $rc; }
step PROF timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o prof -- python bench.py --no-cpu > gpurun_out/prof_$TAG.log 2>&1
python scripts/kstats.py gpurun_out/prof_$TAG > gpurun_out/kstats_$TAG.txt
step SER env AMD_SERIALIZE_KERNEL=3 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ser_$TAG -o prof -- python bench.py --steps 2 --warmup 1 --no-cpu > gpurun_out/ser_$TAG.log 2>&1
python scripts/kstats.py gpurun_out/ser_$TAG > gpurun_out/kstats_ser_$TAG.txt
cat gpurun_out/kstats_$TAG.txt gpurun_out/kstats_ser_$TAG.txt | head -70
