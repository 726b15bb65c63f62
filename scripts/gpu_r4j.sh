#!/bin/bash
# Round 4: kernel trace of the world-8 owner-shaped shard build (12.5M records) on one GPU.
export TMPDIR=/tmp
TAG=${1:-r4j}
step() { local name=$1; shift; "$@"; local rc=$?; echo "${name}_RC=$rc" >&2; [ $rc -eq 0 ] || exit $rc; }
step SIM timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/sim_$TAG -o sim -- python3 scripts/shard_rank_sim.py --world 8 > gpurun_out/sim_$TAG.json 2> gpurun_out/sim_$TAG.err
cut -c1-600 gpurun_out/sim_$TAG.json
