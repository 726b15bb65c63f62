#!/bin/bash
# Small levels read the leaf stashes themselves (no per-level leaf-record pass): GPU suite, then
# a same-box A/B against the HEAD build (scripts/build_ab_base.sh) at 100M and in the world-8 sim
export TMPDIR=/tmp
tag=${1:-r4ak}
step() { local name=$1; shift; "$@"; local rc=$?; echo "${name}_RC=$rc" >&2; [ $rc -eq 0 ] || exit $rc; }
step PYTEST timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 200 --timeout-method thread -o log_cli=false > gpurun_out/${tag}_pytest.log 2>&1
tail -3 gpurun_out/${tag}_pytest.log
step AB bash scripts/gpu_ab_lib.sh $tag "base:KHST_LIB_AB=khipu_amd/libkhst_base.so" "new:X=1"
for rep in 1 2; do
  step SIMB timeout -k 10 300 env KHST_LIB_AB=khipu_amd/libkhst_base.so python3 scripts/shard_rank_sim.py --world 8 > gpurun_out/${tag}_sim_base_$rep.json 2>/dev/null
  step SIMN timeout -k 10 300 python3 scripts/shard_rank_sim.py --world 8 > gpurun_out/${tag}_sim_new_$rep.json 2>/dev/null
  python3 -c "import json;[print(f, json.load(open('gpurun_out/${tag}_sim_'+f+'_$rep.json')).get('ms_per_step')) for f in ('base','new')]"
done
echo done
