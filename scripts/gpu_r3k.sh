#!/bin/bash
# round 3: where k_leaf_in's cycles go (one PMC pass: SQ counters only), beside key hashing
export TMPDIR=/tmp
tag=${1:-r3k}
timeout -s KILL 150 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_LDS --output-format csv -d gpurun_out/pmc_$tag -o pmc -- python3 bench.py --accounts 100000000 --steps 1 --warmup 1 --no-cpu > gpurun_out/pmc_$tag.log 2>&1
echo PMC_RC=$?
