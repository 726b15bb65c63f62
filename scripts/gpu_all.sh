#!/bin/bash
# the whole GPU suite, the block-commit trace at 50M, configs[1..3], the owner-shaped shard
# simulation at N = 2, 4, 8 and the list-roots line
export TMPDIR=/tmp
tag=${1:-all}
step() { local name=$1; shift; "$@"; local rc=$?; echo "${name}_RC=$rc" >&2; [ $rc -eq 0 ] || exit $rc; }
step PYTEST timeout -k 10 700 python -u -m pytest tests -x -v -m gpu --timeout 200 --timeout-method thread -o log_cli=false > gpurun_out/pytest_$tag.log 2>&1
tail -2 gpurun_out/pytest_$tag.log
step BC timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/bc_$tag -o bc -- python3 scripts/block_commit_prof.py > gpurun_out/bc_$tag.log 2>&1
grep block_wall gpurun_out/bc_$tag.log
python3 scripts/block_trace.py gpurun_out/bc_$tag --timeline gpurun_out/bc_timeline_$tag.json > gpurun_out/bc_trace_$tag.json && head -6 gpurun_out/bc_trace_$tag.json
step CONFIGS timeout -k 10 600 python scripts/bench_configs.py --cfg 2 4 3 > gpurun_out/configs_$tag.jsonl 2> gpurun_out/configs_$tag.err
cut -c1-300 gpurun_out/configs_$tag.jsonl
for w in 2 4 8; do
  step SIM$w timeout -k 10 300 python3 scripts/shard_rank_sim.py --world $w > gpurun_out/sim_${tag}_w$w.json 2> gpurun_out/sim_${tag}_w$w.err
  cut -c1-300 gpurun_out/sim_${tag}_w$w.json
done
step LISTS timeout -k 10 300 python bench.py --workload lists > gpurun_out/bench_lists_$tag.json 2> gpurun_out/bench_lists_$tag.err
cut -c1-300 gpurun_out/bench_lists_$tag.json
