#!/bin/bash
# Two-pass parent-depth scatter (k_pd2_*: KHST_TOPO_TILE=4 after the tile kernel, =5 first):
# switch parity tests, then the 100M step against the default (=1, scatter folded into the
# tile kernel) and the world-8 simulation
export TMPDIR=/tmp
tag=${1:-r4be}
step() { local name=$1; shift; "$@"; local rc=$?; echo "${name}_RC=$rc" >&2; [ $rc -eq 0 ] || exit $rc; }
step PYTEST timeout -k 10 600 python -u -m pytest tests/test_gpu_switches.py -x -q -m gpu -k "TOPO_TILE" --timeout 200 --timeout-method thread -o log_cli=false > gpurun_out/${tag}_pytest.log 2>&1
grep -E "passed|failed" gpurun_out/${tag}_pytest.log | tail -1
step AB bash scripts/gpu_ab_lib.sh $tag "t1:KHST_TOPO_TILE=1" "t4:KHST_TOPO_TILE=4"
step TRACE timeout -k 10 300 env KHST_TOPO_TILE=4 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${tag}_tr -o tr -- python3 bench.py --steps 3 --warmup 1 --no-cpu --no-host-path > gpurun_out/${tag}_tr.json 2>/dev/null
echo done
