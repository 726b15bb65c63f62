#!/bin/bash
# k_branch_small's level cap (KHST_SMALL_LEVEL, default 32768) raised over the 65k / 131k
# full-branch levels: 100M step and the world-8 simulation, alternated on one box
export TMPDIR=/tmp
tag=${1:-r4an}
step() { local name=$1; shift; "$@"; local rc=$?; echo "${name}_RC=$rc" >&2; [ $rc -eq 0 ] || exit $rc; }
step AB bash scripts/gpu_ab_lib.sh $tag "def:X=1" "s140k:KHST_SMALL_LEVEL=140000" "s70k:KHST_SMALL_LEVEL=70000"
for rep in 1 2; do
  for v in def:X=1 s140k:KHST_SMALL_LEVEL=140000 s70k:KHST_SMALL_LEVEL=70000; do
    l=${v%%:*}; e=${v#*:}
    step SIM_$l timeout -k 10 300 env $e python3 scripts/shard_rank_sim.py --world 8 > gpurun_out/${tag}_sim_${l}_$rep.json 2>/dev/null
    python3 -c "import json;d=json.load(open('gpurun_out/${tag}_sim_${l}_$rep.json'));print('$l', d['ms']['build'], d['critical_path_ms_excl_exchange'], d['build_stages_ms']['branches'])"
  done
done
echo done
