#!/bin/bash
# Round 4: the drop-in host path at 100M (bench.py, no CPU legs) and the f3 verify workload.
export TMPDIR=/tmp
TAG=${1:-r4e}
step() { local name=$1; shift; "$@"; local rc=$?; echo "${name}_RC=$rc" >&2; [ $rc -eq 0 ] || exit $rc; }
step VERIFY timeout -k 10 400 python bench.py --workload verify --steps 5 --warmup 2 > gpurun_out/bench_verify_$TAG.json 2> gpurun_out/bench_verify_$TAG.err
cut -c1-600 gpurun_out/bench_verify_$TAG.json
step BENCH timeout -k 10 400 python bench.py --steps 5 --warmup 2 --no-cpu > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
python -c "import json;d=json.load(open('gpurun_out/bench_$TAG.json'));print(d['ms_per_step'], d['drop_in_host_path'])"
