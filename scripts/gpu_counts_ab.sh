#!/bin/bash
# forest commit without the op-count sync (buffers sized by bounds, the counts read on the
# device and brought back with the gather sync): the whole GPU suite, then configs[2] at 50M
# alternated with the HEAD build (the variant is khipu_amd/libkhst_new.so, loaded by KHST_LIB_AB)
export TMPDIR=/tmp
tag=${1:-cs}
step() { local name=$1; shift; "$@"; local rc=$?; echo "${name}_RC=$rc" >&2; [ $rc -eq 0 ] || exit $rc; }
step PYTEST env KHST_LIB_AB=khipu_amd/libkhst_new.so timeout -k 10 700 python -u -m pytest tests -x -q -m gpu --timeout 200 --timeout-method thread -o log_cli=false > gpurun_out/pytest_$tag.log 2>&1
tail -1 gpurun_out/pytest_$tag.log
for v in new base new2 base2; do
  case $v in
    new*) envs="KHST_LIB_AB=khipu_amd/libkhst_new.so" ;;
    base*) envs="KHST_AB=none" ;;
  esac
  step CFG2_$v env $envs timeout -k 10 400 python scripts/bench_configs.py --cfg 3 --no-cpu > gpurun_out/cfg2_${tag}_$v.jsonl 2> gpurun_out/cfg2_${tag}_$v.err
  python -c "import json;d=json.loads(open('gpurun_out/cfg2_${tag}_$v.jsonl').readline());print('$v', round(d['block_ms_median'],3), [round(x,3) for x in d['block_ms_all']])"
done
