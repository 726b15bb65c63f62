#!/bin/bash
# Round-end evidence, part B: PMC passes at 100M, FETCH/WRITE_SIZE calibration, the sharded
# world-1 line, the secondary configs, the list-roots workload.
export TMPDIR=/tmp
TAG=${1:-r2z}
step() { local name=$1; shift; "$@"; local rc=$?; echo "${name}_RC=$rc" >&2; [ $rc -eq 0 ] || exit $rc; }
step PMC bash scripts/gpu_pmc.sh ${TAG}pmc
python scripts/pmc_summary.py ${TAG}pmc --json gpurun_out/${TAG}_pmc_traffic_100000000.json > gpurun_out/${TAG}_pmc_summary.txt
head -30 gpurun_out/${TAG}_pmc_summary.txt
step CALIB bash scripts/gpu_calib.sh
step SHARDED timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 1 --sharded --steps 3 --warmup 1 --seq-samples 20000 > gpurun_out/bench_sh_$TAG.json 2> gpurun_out/bench_sh_$TAG.err
cut -c1-400 gpurun_out/bench_sh_$TAG.json
step LISTS timeout -k 10 300 python bench.py --workload lists > gpurun_out/bench_lists_$TAG.json 2> gpurun_out/bench_lists_$TAG.err
cut -c1-600 gpurun_out/bench_lists_$TAG.json
step CONFIGS timeout -k 10 600 python scripts/bench_configs.py --cfg 2 4 3 > gpurun_out/configs_$TAG.jsonl 2> gpurun_out/configs_$TAG.err
cut -c1-500 gpurun_out/configs_$TAG.jsonl
