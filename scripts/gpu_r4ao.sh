#!/bin/bash
# Owner partition with the value bytes per owner summed in the count pass (the length scan
# after the counts are back): partition / sharded GPU tests, then the world-8 simulation
# alternated with the HEAD build (scripts/build_ab_base.sh)
export TMPDIR=/tmp
tag=${1:-r4ao}
step() { local name=$1; shift; "$@"; local rc=$?; echo "${name}_RC=$rc" >&2; [ $rc -eq 0 ] || exit $rc; }
step PYTEST timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_sharded_cabi.py tests/test_gpu_sharded_torch.py -x -q -m gpu --timeout 200 --timeout-method thread -o log_cli=false > gpurun_out/${tag}_pytest.log 2>&1
step TRACE timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${tag}_tr -o tr -- python3 scripts/shard_rank_sim.py --world 8 --steps 3 > gpurun_out/${tag}_tr.json 2>/dev/null
tail -1 gpurun_out/${tag}_pytest.log
for rep in 1 2; do
  for v in new base; do
    case $v in
      new) e="X=1" ;;
      base) e="KHST_LIB_AB=khipu_amd/libkhst_base.so" ;;
    esac
    step SIM_$v timeout -k 10 300 env $e python3 scripts/shard_rank_sim.py --world 8 > gpurun_out/${tag}_sim_${v}_$rep.json 2>/dev/null
    python3 -c "import json;d=json.load(open('gpurun_out/${tag}_sim_${v}_$rep.json'));print('$v', d['ms'], d['critical_path_ms_excl_exchange'])"
  done
done
echo done
