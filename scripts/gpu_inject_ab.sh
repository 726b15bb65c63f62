#!/bin/bash
# block commit with the injection's error word read at the account commit's first sync (one
# host sync less per block): resident + configs tests, then configs[2] at 50M alternated with
# the HEAD build (KHST_LIB_AB, scripts/build_ab_base.sh)
export TMPDIR=/tmp
tag=${1:-ij}
step() { local name=$1; shift; "$@"; local rc=$?; echo "${name}_RC=$rc" >&2; [ $rc -eq 0 ] || exit $rc; }
step PYTEST timeout -k 10 400 python -u -m pytest tests/test_gpu_resident.py tests/test_gpu_configs.py -x -q -m gpu --timeout 200 --timeout-method thread -o log_cli=false > gpurun_out/pytest_$tag.log 2>&1
tail -1 gpurun_out/pytest_$tag.log
for v in new base new2 base2; do
  case $v in
    new*) envs="KHST_AB=none" ;;
    base*) envs="KHST_LIB_AB=khipu_amd/libkhst_base.so" ;;
  esac
  step CFG2_$v env $envs timeout -k 10 400 python scripts/bench_configs.py --cfg 3 --no-cpu > gpurun_out/cfg2_${tag}_$v.jsonl 2> gpurun_out/cfg2_${tag}_$v.err
  python -c "import json;d=json.loads(open('gpurun_out/cfg2_${tag}_$v.jsonl').readline());print('$v', round(d['block_ms_median'],3), [round(x,3) for x in d['block_ms_all']])"
done
