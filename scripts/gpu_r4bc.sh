#!/bin/bash
# k_branch_xl: the extension hashed lane-spread (r4bc) and the publish context loaded up front (r4bd):
# GPU suite, then configs[2] block commits, the world-8 simulation and the 100M step, alternated
# with the HEAD build (scripts/build_ab_base.sh)
export TMPDIR=/tmp
tag=${1:-r4bc}
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
  step SIM_$v timeout -k 10 300 env $e python3 scripts/shard_rank_sim.py --world 8 > gpurun_out/${tag}_sim_$v.json 2>/dev/null
  python3 -c "import json;d=json.load(open('gpurun_out/${tag}_sim_$v.json'));print('$v sim', d['ms']['build'], d['critical_path_ms_excl_exchange'], d['build_stages_ms']['branches'])"
done
step AB bash scripts/gpu_ab_lib.sh $tag "base:KHST_LIB_AB=khipu_amd/libkhst_base.so" "new:X=1"
echo done
