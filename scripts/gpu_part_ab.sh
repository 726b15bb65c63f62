#!/bin/bash
# partition A/B (16-byte key moves in k_part_place): the partition parity tests, then the
# world-8 per-rank simulation with the new library and the HEAD build, alternated
export TMPDIR=/tmp
tag=${1:-pt}
step() { local name=$1; shift; "$@"; local rc=$?; echo "${name}_RC=$rc" >&2; [ $rc -eq 0 ] || exit $rc; }
step PYTEST timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_sharded_cabi.py tests/test_gpu_sharded_torch.py -x -q -m gpu --timeout 200 --timeout-method thread -o log_cli=false > gpurun_out/pytest_$tag.log 2>&1
tail -1 gpurun_out/pytest_$tag.log
for v in new base new2 base2; do
  case $v in
    new*) envs="KHST_AB=none" ;;
    base*) envs="KHST_LIB_AB=khipu_amd/libkhst_base.so" ;;
  esac
  step SIM_$v env $envs timeout -k 10 300 python scripts/shard_rank_sim.py --world 8 > gpurun_out/sim_${tag}_$v.json 2> gpurun_out/sim_${tag}_$v.err
  python -c "import json;d=json.load(open('gpurun_out/sim_${tag}_$v.json'));print('$v', d['ms'])"
done
