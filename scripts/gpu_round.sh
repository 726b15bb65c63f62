#!/bin/bash
# One GPU verification round: parity tests, rocprofv3 kernel stats, bench (single + sharded path).
# Every GPU step has its own time limit; the first failing step ends the round.
export TMPDIR=/tmp
TAG=${1:-r}
step() { local name=$1; shift; "$@"; local rc=$?; echo "${name}_RC=$rc" >&2; [ $rc -eq 0 ] || exit $rc; }
step SMOKE timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/smoke_$TAG.log 2>&1
step PYTEST timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread -o log_cli=false --junitxml=gpurun_out/pytest_$TAG.xml > gpurun_out/pytest_$TAG.log 2>&1
tail -3 gpurun_out/pytest_$TAG.log
step PROF timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o prof -- python bench.py --accounts ${PROF_ACCOUNTS:-10000000} --steps 3 --warmup 1 --no-cpu > gpurun_out/prof_$TAG.log 2>&1
step BENCH timeout -k 10 600 python bench.py --accounts ${BENCH_ACCOUNTS:-100000000} --steps 5 --warmup 2 > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
cat gpurun_out/bench_$TAG.json
if [ -z "$NO_SHARDED" ]; then
step SHARDED timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 1 --sharded --accounts ${BENCH_ACCOUNTS:-100000000} --steps 3 --warmup 1 --seq-samples 20000 > gpurun_out/bench_sh_$TAG.json 2> gpurun_out/bench_sh_$TAG.err
cat gpurun_out/bench_sh_$TAG.json
fi
