#!/bin/bash
# sharded-path checks on one GPU: GPU tests for the partition / late values / RCCL world 1,
# the per-rank simulation at N = 2, 4, 8, and the world-1 sharded bench
export TMPDIR=/tmp
tag=${1:-x}
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_parity.py -m gpu \
  -k "partition or late_values or rccl_world1 or sharded" > gpurun_out/shard_pytest_$tag.log 2>&1 || { tail -30 gpurun_out/shard_pytest_$tag.log; exit 1; }
tail -2 gpurun_out/shard_pytest_$tag.log
for w in 2 4 8; do
  timeout -k 10 300 python scripts/shard_rank_sim.py --world $w > gpurun_out/shard_sim_${tag}_$w.json || exit 1
  cat gpurun_out/shard_sim_${tag}_$w.json
done
timeout -k 10 300 python bench.py --sharded --steps 5 --warmup 2 --no-cpu > gpurun_out/shard_bench_$tag.json 2> gpurun_out/shard_bench_$tag.err || { tail gpurun_out/shard_bench_$tag.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/shard_bench_$tag.json'));print(d['ms_per_step'], d['state_root'][:12], d['phase_ms_max_over_ranks'])"
