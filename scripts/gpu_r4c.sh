#!/bin/bash
# Round 4: the grouped build A/B at 100M (KHST_GROUPS = 1 / 2 / 4 / 8, roots must agree), then the
# grouped / versioned / resident / configs GPU tests.  Each GPU step has its own limit.
export TMPDIR=/tmp
TAG=${1:-r4c}
step() { local name=$1; shift; "$@"; local rc=$?; echo "${name}_RC=$rc" >&2; [ $rc -eq 0 ] || exit $rc; }
for G in ${GROUPS_AB:-1 4 2 8}; do
  step BENCH_G$G timeout -k 10 300 env KHST_GROUPS=$G python bench.py --steps 5 --warmup 2 --no-cpu > gpurun_out/bench_${TAG}_g$G.json 2> gpurun_out/bench_${TAG}_g$G.err
  python -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[2],round(d['ms_per_step'],2),d['state_root'][:16],d['stage_ms'],d['roofline']['frac'])" gpurun_out/bench_${TAG}_g$G.json G$G
done
step PYTEST timeout -k 10 900 python -u -m pytest ${TESTS:-tests/test_gpu_grouped.py tests/test_gpu_versioned.py tests/test_gpu_resident.py tests/test_gpu_configs.py} -x -v -m gpu --timeout 300 --timeout-method thread -o log_cli=false > gpurun_out/pytest_$TAG.log 2>&1
tail -5 gpurun_out/pytest_$TAG.log
