#!/bin/bash
# Instruction-cache and issue counters over one 100M bench step (one rocprofv3 run per pass)
export TMPDIR=/tmp
TAG=${1:-ic}
N=${PMC_ACCOUNTS:-100000000}
run() {
  local p=$1; shift
  timeout -s KILL 240 rocprofv3 --kernel-trace --pmc "$@" --output-format csv -d gpurun_out/${TAG}_$p -o pmc \
    -- python3 bench.py --accounts $N --steps 1 --warmup 1 --no-cpu --no-host-path > gpurun_out/${TAG}_$p.log 2>&1
  local rc=$?; echo "PMC_${p}_RC=$rc"; [ $rc -eq 0 ] || exit $rc
}
run p1 SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE
run p2 SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_BRANCH SQ_INSTS_SALU SQ_IFETCH SQ_INSTS_VALU SQ_WAIT_ANY SQ_BUSY_CYCLES
