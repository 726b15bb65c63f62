#!/bin/bash
export TMPDIR=/tmp
set -o pipefail
bash scripts/gpu_tests.sh r2e -k "configs or resident or forest" && \
timeout -k 10 600 python scripts/bench_configs.py --cfg 3 --steps 5 --warmup 1 > gpurun_out/cfg3_r2e.json 2> gpurun_out/cfg3_r2e.err; rc=$?; cat gpurun_out/cfg3_r2e.json; tail -5 gpurun_out/cfg3_r2e.err; exit $rc
