#!/bin/bash
# Full GPU suite at HEAD + the world-8 simulation (3 runs)
export TMPDIR=/tmp
tag=${1:-r4ar}
step() { local name=$1; shift; "$@"; local rc=$?; echo "${name}_RC=$rc" >&2; [ $rc -eq 0 ] || exit $rc; }
step PYTEST timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 200 --timeout-method thread -o log_cli=false > gpurun_out/${tag}_pytest.log 2>&1
grep -E "passed|failed" gpurun_out/${tag}_pytest.log | tail -1
for rep in 1 2 3; do
  step SIM timeout -k 10 300 python3 scripts/shard_rank_sim.py --world 8 > gpurun_out/${tag}_sim_$rep.json 2>/dev/null
  python3 -c "import json;d=json.load(open('gpurun_out/${tag}_sim_$rep.json'));print(d['ms'], d['critical_path_ms_excl_exchange'], d['build_stages_ms'])"
done
echo done
