#!/bin/bash
# round 3: block-commit kernel trace at 50M (configs[2]), owner-shaped shard simulation at
# N = 2, 4, 8, the storage line with per-step device times
export TMPDIR=/tmp
tag=${1:-r3h}
step() { local name=$1; shift; "$@"; local rc=$?; echo "${name}_RC=$rc" >&2; [ $rc -eq 0 ] || exit $rc; }
step BC timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/bc_$tag -o bc -- python3 scripts/block_commit_prof.py > gpurun_out/bc_$tag.log 2>&1
tail -1 gpurun_out/bc_$tag.log
python3 scripts/block_trace.py gpurun_out/bc_$tag > gpurun_out/bc_trace_$tag.json && head -60 gpurun_out/bc_trace_$tag.json
for w in 2 4 8; do
  step SIM$w timeout -k 10 300 python3 scripts/shard_rank_sim.py --world $w > gpurun_out/sim_${tag}_w$w.json 2> gpurun_out/sim_${tag}_w$w.err
  cat gpurun_out/sim_${tag}_w$w.json
done
step STORAGE timeout -k 10 300 python bench.py --workload storage --steps 5 --warmup 2 --no-cpu > gpurun_out/storage_$tag.json 2> gpurun_out/storage_$tag.err
python -c "import json; d=json.load(open('gpurun_out/storage_$tag.json')); print(d['ms_per_step'], d['rank0_device_ms_per_step'])"
