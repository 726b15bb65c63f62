#!/bin/bash
# lane-spread Keccak (keccak_xlane.h): equality + latency check, the whole GPU suite, the
# block-commit trace at 50M, the configs[2] line and the default 100M bench
export TMPDIR=/tmp
tag=${1:-xl}
step() { local name=$1; shift; "$@"; local rc=$?; echo "${name}_RC=$rc" >&2; [ $rc -eq 0 ] || exit $rc; }
step XLCHECK timeout -k 10 60 scripts/xlane_check > gpurun_out/xlane_$tag.json
cat gpurun_out/xlane_$tag.json
step PYTEST timeout -k 10 700 python -u -m pytest tests -x -v -m gpu --timeout 200 --timeout-method thread -o log_cli=false > gpurun_out/pytest_$tag.log 2>&1
tail -2 gpurun_out/pytest_$tag.log
step BC timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/bc_$tag -o bc -- python3 scripts/block_commit_prof.py > gpurun_out/bc_$tag.log 2>&1
grep block_wall gpurun_out/bc_$tag.log
python3 scripts/block_trace.py gpurun_out/bc_$tag --timeline gpurun_out/bc_timeline_$tag.json > gpurun_out/bc_trace_$tag.json && head -12 gpurun_out/bc_trace_$tag.json
step CFG2 timeout -k 10 400 python scripts/bench_configs.py --cfg 3 > gpurun_out/cfg2_$tag.jsonl 2> gpurun_out/cfg2_$tag.err
cut -c180-330 gpurun_out/cfg2_$tag.jsonl
step BENCH timeout -k 10 600 python bench.py --no-cpu > gpurun_out/bench_$tag.json 2> gpurun_out/bench_$tag.err
cut -c1-700 gpurun_out/bench_$tag.json
step API timeout -k 10 400 rocprofv3 --kernel-trace --hip-trace --output-format csv -d gpurun_out/bca_$tag -o bca -- python3 scripts/block_commit_prof.py > gpurun_out/bca_$tag.log 2>&1
python3 scripts/api_trace.py gpurun_out/bca_$tag > gpurun_out/api_$tag.json && head -60 gpurun_out/api_$tag.json
