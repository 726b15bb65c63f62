#!/bin/bash
# refresh of the secondary configs after the small-level kernels: configs[1..3]
# (scripts/bench_configs.py), the owner-shaped shard simulation at N = 2, 4, 8, list roots
export TMPDIR=/tmp
tag=${1:-cfg}
step() { local name=$1; shift; "$@"; local rc=$?; echo "${name}_RC=$rc" >&2; [ $rc -eq 0 ] || exit $rc; }
step XLT timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -k lane_spread -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/xlt_$tag.log 2>&1
tail -1 gpurun_out/xlt_$tag.log
step CONFIGS timeout -k 10 600 python scripts/bench_configs.py --cfg 2 4 3 > gpurun_out/configs_$tag.jsonl 2> gpurun_out/configs_$tag.err
cut -c1-300 gpurun_out/configs_$tag.jsonl
for w in 2 4 8; do
  step SIM$w timeout -k 10 300 python3 scripts/shard_rank_sim.py --world $w > gpurun_out/sim_${tag}_w$w.json 2> gpurun_out/sim_${tag}_w$w.err
  cut -c1-400 gpurun_out/sim_${tag}_w$w.json
done
step LISTS timeout -k 10 300 python bench.py --workload lists > gpurun_out/bench_lists_$tag.json 2> gpurun_out/bench_lists_$tag.err
cut -c1-300 gpurun_out/bench_lists_$tag.json
