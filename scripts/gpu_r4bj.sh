#!/bin/bash
# Late account leaves listed in the first leaf pass and hashed by the second (no full sweep,
# no hash launch after it): GPU suite, configs[2] A/B against the HEAD build, kernel traces
export TMPDIR=/tmp
tag=${1:-r4bh}
step() { local name=$1; shift; "$@"; local rc=$?; echo "${name}_RC=$rc" >&2; [ $rc -eq 0 ] || exit $rc; }
step PYTEST timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 200 --timeout-method thread -o log_cli=false > gpurun_out/${tag}_pytest.log 2>&1
grep -E "passed|failed" gpurun_out/${tag}_pytest.log | tail -1
for v in new base new2 base2; do
  case $v in
    new*) e="X=1" ;;
    base*) e="KHST_LIB_AB=khipu_amd/libkhst_base.so" ;;
  esac
  step CFG2_$v env $e timeout -k 10 400 python scripts/bench_configs.py --cfg 3 --no-cpu > gpurun_out/${tag}_cfg2_$v.jsonl 2> gpurun_out/${tag}_cfg2_$v.err
  python -c "import json;d=json.loads(open('gpurun_out/${tag}_cfg2_$v.jsonl').readline());print('$v', round(d['block_ms_median'],3), [round(x,3) for x in d['block_ms_all']])"
done
export KHST_LIB_AB=khipu_amd/libkhst.so
step TRACE_new timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${tag}_bc_new -o bc -- python3 scripts/block_commit_prof.py > gpurun_out/${tag}_bc_new.log 2>&1
export KHST_LIB_AB=khipu_amd/libkhst_base.so
step TRACE_base timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${tag}_bc_base -o bc -- python3 scripts/block_commit_prof.py > gpurun_out/${tag}_bc_base.log 2>&1
echo done
