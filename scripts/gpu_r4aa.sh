#!/bin/bash
# Round 4: block commit with the storage roots injected right after the storage element build
# (FCommit::after_roots): GPU suite, then configs[2] at 50M twice
export TMPDIR=/tmp
tag=${1:-r4aa}
step() { local name=$1; shift; "$@"; local rc=$?; echo "${name}_RC=$rc" >&2; [ $rc -eq 0 ] || exit $rc; }
step PYTEST timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_${tag}.log 2>&1
tail -1 gpurun_out/pytest_${tag}.log
for v in a b; do
  step CFG3_$v timeout -k 10 300 python scripts/bench_configs.py --cfg 3 --no-cpu > gpurun_out/cfg3_${tag}_$v.json 2> gpurun_out/cfg3_${tag}_$v.err
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], round(d['block_ms_median'],3), [round(x,3) for x in d['block_ms_all']])" gpurun_out/cfg3_${tag}_$v.json $v
done
