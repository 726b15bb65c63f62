#!/bin/bash
# Round-end evidence, part B: PMC passes at 100M, the sharded world-1 line, the list-roots
# and storage-trie workloads, the secondary configs.  (The FETCH/WRITE_SIZE calibration,
# scripts/gpu_calib.sh, is per access shape and kept from round 2.)
export TMPDIR=/tmp
TAG=${1:-r2z}
step() { local name=$1; shift; "$@"; local rc=$?; echo "${name}_RC=$rc" >&2; [ $rc -eq 0 ] || exit $rc; }
step PMC bash scripts/gpu_pmc.sh ${TAG}pmc
python scripts/pmc_summary.py ${TAG}pmc --json gpurun_out/${TAG}_pmc_traffic_100000000.json > gpurun_out/${TAG}_pmc_summary.txt
head -30 gpurun_out/${TAG}_pmc_summary.txt
step SHARDED timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 1 --sharded --steps 3 --warmup 1 --seq-samples 20000 > gpurun_out/bench_sh_$TAG.json 2> gpurun_out/bench_sh_$TAG.err
cut -c1-400 gpurun_out/bench_sh_$TAG.json
step LISTS timeout -k 10 300 python bench.py --workload lists > gpurun_out/bench_lists_$TAG.json 2> gpurun_out/bench_lists_$TAG.err
cut -c1-600 gpurun_out/bench_lists_$TAG.json
step STORAGE timeout -k 10 300 python bench.py --workload storage > gpurun_out/bench_storage_$TAG.json 2> gpurun_out/bench_storage_$TAG.err
cut -c1-600 gpurun_out/bench_storage_$TAG.json
step CONFIGS timeout -k 10 600 python scripts/bench_configs.py --cfg 2 4 3 > gpurun_out/configs_$TAG.jsonl 2> gpurun_out/configs_$TAG.err
cut -c1-500 gpurun_out/configs_$TAG.jsonl
