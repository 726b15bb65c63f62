#!/bin/bash
# Kernel trace of the world-8 shard simulation (scripts/shard_rank_sim.py): where one rank's
# hash / partition / build time goes
export TMPDIR=/tmp
tag=${1:-r4am}
step() { local name=$1; shift; "$@"; local rc=$?; echo "${name}_RC=$rc" >&2; [ $rc -eq 0 ] || exit $rc; }
step TRACE timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/${tag}_sim -o sim -- python3 scripts/shard_rank_sim.py --world 8 --steps 3 > gpurun_out/${tag}_sim.json 2> gpurun_out/${tag}_sim.err
cut -c1-300 gpurun_out/${tag}_sim.json
echo done
