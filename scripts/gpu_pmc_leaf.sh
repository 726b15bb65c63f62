#!/bin/bash
# one extra PMC pass (measurement only): instruction mix and wait cycles of the hash kernels
export TMPDIR=/tmp
timeout -s KILL 150 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES --output-format csv -d gpurun_out/pmcleaf -o pmc -- python3 bench.py --accounts 100000000 --steps 1 --warmup 1 --no-cpu > gpurun_out/pmcleaf.log 2>&1
echo PMC_RC=$?
