#!/bin/bash
# leaf positions (trie_ops.h Topo::lpos): the whole GPU suite, then the 100M bench A/B
# against the copy pass (KHST_LEAF_POS=0), alternated, and the step's kernel timeline
export TMPDIR=/tmp
tag=${1:-lp}
step() { local name=$1; shift; "$@"; local rc=$?; echo "${name}_RC=$rc" >&2; [ $rc -eq 0 ] || exit $rc; }
step PYTEST timeout -k 10 700 python -u -m pytest tests -x -v -m gpu --timeout 200 --timeout-method thread -o log_cli=false > gpurun_out/pytest_$tag.log 2>&1
tail -2 gpurun_out/pytest_$tag.log
for v in pos move pos2 move2; do
  case $v in
    pos*) envs="KHST_LEAF_POS=1" ;;
    move*) envs="KHST_LEAF_POS=0" ;;
  esac
  step BENCH_$v env $envs timeout -k 10 300 python bench.py --no-cpu > gpurun_out/bench_${tag}_$v.json 2> gpurun_out/bench_${tag}_$v.err
  cut -c1-420 gpurun_out/bench_${tag}_$v.json
done
step ST timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/st_$tag -o st -- python3 bench.py --steps 2 --warmup 1 --no-cpu > gpurun_out/st_$tag.log 2>&1
python3 scripts/step_timeline.py gpurun_out/st_$tag > gpurun_out/step_timeline_$tag.json && cut -c1-600 gpurun_out/step_timeline_$tag.json
