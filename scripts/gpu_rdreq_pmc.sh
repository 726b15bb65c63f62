#!/bin/bash
# HBM read requests by size over one 100M bench step (2 builds): bytes = 32 x RDREQ_32B +
# 64 x RDREQ_64B + 128 x RDREQ_128B, a cross-check of the 2 x FETCH_SIZE convention per kernel
export TMPDIR=/tmp
TAG=${1:-rq}
N=${PMC_ACCOUNTS:-100000000}
run() {
  local p=$1; shift
  timeout -s KILL 240 rocprofv3 --kernel-trace --pmc "$@" --output-format csv -d gpurun_out/${TAG}_$p -o pmc \
    -- python3 bench.py --accounts $N --steps 1 --warmup 1 --no-cpu --no-host-path > gpurun_out/${TAG}_$p.log 2>&1
  local rc=$?; echo "PMC_${p}_RC=$rc"; [ $rc -eq 0 ] || exit $rc
}
run p1 TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum
run p2 FETCH_SIZE
