#!/bin/bash
# round 3: key hashing with the owner count folded in (kh_dev_hash_partition_ev) -- parity
# against the oracle's kec256 + a stable host partition, then the per-rank simulation at
# N = 2, 4, 8 with the fused and the separate calls timed side by side
export TMPDIR=/tmp
tag=${1:-r3t}
step() { local name=$1; shift; "$@"; local rc=$?; echo "${name}_RC=$rc" >&2; [ $rc -eq 0 ] || exit $rc; }
step PYTEST timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "partition" -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_$tag.log 2>&1
tail -1 gpurun_out/pytest_$tag.log
for w in 2 4 8; do
  step SIM$w timeout -k 10 300 python3 scripts/shard_rank_sim.py --world $w > gpurun_out/sim_${tag}_w$w.json 2> gpurun_out/sim_${tag}_w$w.err
  cat gpurun_out/sim_${tag}_w$w.json
done
