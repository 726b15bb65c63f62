#!/bin/bash
# PMC passes over one bench step (1 warmup + 1 timed build), one rocprofv3 run per
# counter group (rocprofv3 does not split counters over passes; FETCH_SIZE uses 3 TCC
# slots and WRITE_SIZE 2, so they take separate passes).  Summarise with
#   python scripts/pmc_summary.py <tag> [--json profiles/<tag>_pmc_traffic.json]
# Every pass has its own time limit; the first failing pass ends the script.
export TMPDIR=/tmp
TAG=${1:-pmc}
N=${PMC_ACCOUNTS:-100000000}
run() {
  local p=$1; shift
  timeout -s KILL 240 rocprofv3 --kernel-trace --pmc "$@" --output-format csv -d gpurun_out/${TAG}_$p -o pmc \
    -- python3 bench.py --accounts $N --steps 1 --warmup 1 --no-cpu --no-host-path > gpurun_out/${TAG}_$p.log 2>&1
  local rc=$?; echo "PMC_${p}_RC=$rc"; [ $rc -eq 0 ] || exit $rc
}
run p1 FETCH_SIZE
run p2 WRITE_SIZE
run p3 SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_WAVES
