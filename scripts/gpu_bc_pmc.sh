#!/bin/bash
# PMC passes over configs[2] block commits (scripts/block_commit_prof.py: 2 warmup + 3 blocks
# on the 50M resident state), one rocprofv3 run per counter group; summarise with
#   python scripts/pmc_summary.py <tag> 5
export TMPDIR=/tmp
TAG=${1:-bcpmc}
run() {
  local p=$1; shift
  timeout -s KILL 400 rocprofv3 --kernel-trace --pmc "$@" --output-format csv -d gpurun_out/${TAG}_$p -o pmc \
    -- python3 scripts/block_commit_prof.py --gap-ms 5 > gpurun_out/${TAG}_$p.log 2>&1
  local rc=$?; echo "PMC_${p}_RC=$rc"; [ $rc -eq 0 ] || exit $rc
}
run p1 FETCH_SIZE
run p2 WRITE_SIZE
run p3 SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_WAVES
