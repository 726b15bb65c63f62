#!/bin/bash
# round 3: the new parity checks (refused value-branch update, config2 injection vs the CPU
# builder), then configs at full size with the CPU batch-builder checks
export TMPDIR=/tmp
tag=${1:-r3b}
timeout -k 10 600 python -u -m pytest tests/test_gpu_resident.py tests/test_gpu_configs.py -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_$tag.log 2>&1 || { tail -40 gpurun_out/pytest_$tag.log; exit 1; }
tail -3 gpurun_out/pytest_$tag.log
timeout -k 10 900 python -u scripts/bench_configs.py --cfg 3 4 > gpurun_out/configs_$tag.jsonl 2> gpurun_out/configs_$tag.err || { tail -20 gpurun_out/configs_$tag.err; exit 1; }
cat gpurun_out/configs_$tag.jsonl
