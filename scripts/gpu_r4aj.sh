#!/bin/bash
# Round 4 final measurement set: the N = 1 bench line (CPU legs, host path), its kernel trace,
# configs[1..3] (scripts/bench_configs.py), lists / storage / verify lines, world-8 simulation
export TMPDIR=/tmp
tag=${1:-r4ay}
step() { local name=$1; shift; "$@"; local rc=$?; echo "${name}_RC=$rc" >&2; [ $rc -eq 0 ] || exit $rc; }
step BENCH timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/${tag}_bench.json 2> gpurun_out/${tag}_bench.err
cut -c1-300 gpurun_out/${tag}_bench.json
step PROF timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${tag}_prof -o run -- python3 bench.py --no-cpu --no-host-path --steps 20 --warmup 5 > gpurun_out/${tag}_prof.json 2> gpurun_out/${tag}_prof.err
step CONFIGS timeout -k 10 900 python scripts/bench_configs.py --cfg 2 4 3 > gpurun_out/${tag}_configs.jsonl 2> gpurun_out/${tag}_configs.err
step LISTS timeout -k 10 300 python bench.py --workload lists > gpurun_out/${tag}_lists.json 2> gpurun_out/${tag}_lists.err
step STORAGE timeout -k 10 300 python bench.py --workload storage > gpurun_out/${tag}_storage.json 2> gpurun_out/${tag}_storage.err
step VERIFY timeout -k 10 300 python bench.py --workload verify > gpurun_out/${tag}_verify.json 2> gpurun_out/${tag}_verify.err
step SIM8 timeout -k 10 300 python3 scripts/shard_rank_sim.py --world 8 > gpurun_out/${tag}_sim8.json 2> gpurun_out/${tag}_sim8.err
echo done
