#!/bin/bash
# Iteration round: GPU parity tests, 100M bench without the CPU legs, rocprofv3 kernel stats.
# Every GPU step has its own time limit; the first failing step ends the round.
export TMPDIR=/tmp
TAG=${1:-q}
step() { local name=$1; shift; "$@"; local rc=$?; echo "${name}_RC=$rc" >&2; [ $rc -eq 0 ] || exit $rc; }
step PYTEST timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread -o log_cli=false ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/pytest_$TAG.log 2>&1
tail -3 gpurun_out/pytest_$TAG.log
step BENCH timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
cat gpurun_out/bench_$TAG.json
step PROF timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o prof -- python bench.py --steps 2 --warmup 1 --no-cpu > gpurun_out/prof_$TAG.log 2>&1
python scripts/kstats.py gpurun_out/prof_$TAG > gpurun_out/kstats_$TAG.txt && cat gpurun_out/kstats_$TAG.txt
