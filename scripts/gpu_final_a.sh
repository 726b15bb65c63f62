#!/bin/bash
# Round-end evidence, part A: smoke, the whole GPU suite, the default bench (CPU legs),
# the rocprofv3 kernel summary of the same command, a serialized (standalone) kernel profile.
export TMPDIR=/tmp
TAG=${1:-r2z}
step() { local name=$1; shift; "$@"; local rc=$?; echo "${name}_RC=$rc" >&2; [ $rc -eq 0 ] || exit $rc; }
step SMOKE timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/smoke_$TAG.log 2>&1
step PYTEST timeout -k 10 700 python -u -m pytest tests -x -v -m gpu --timeout 200 --timeout-method thread -o log_cli=false > gpurun_out/pytest_$TAG.log 2>&1
tail -2 gpurun_out/pytest_$TAG.log
step BENCH timeout -k 10 600 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
cat gpurun_out/bench_$TAG.json | cut -c1-600
step PROF timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o prof -- python bench.py --no-cpu > gpurun_out/prof_$TAG.log 2>&1
python scripts/kstats.py gpurun_out/prof_$TAG > gpurun_out/kstats_$TAG.txt
step SER env AMD_SERIALIZE_KERNEL=3 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ser_$TAG -o prof -- python bench.py --steps 2 --warmup 1 --no-cpu > gpurun_out/ser_$TAG.log 2>&1
python scripts/kstats.py gpurun_out/ser_$TAG > gpurun_out/kstats_ser_$TAG.txt
cat gpurun_out/kstats_$TAG.txt gpurun_out/kstats_ser_$TAG.txt | head -70
