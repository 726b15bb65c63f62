#!/bin/bash
# round 3: the 32-bit leaf assembly (k_leaf_in, op_leaf_in3) -- parity, A/B against the
# round-2 kernel (KHST_LEAF=v2) at 100M, and the VALU instruction count per wave
export TMPDIR=/tmp
tag=${1:-r3c}
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_lists.py tests/test_gpu_configs.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_$tag.log 2>&1 || { tail -40 gpurun_out/pytest_$tag.log; exit 1; }
tail -2 gpurun_out/pytest_$tag.log
bash scripts/gpu_ab_lib.sh $tag "v3:X=1" "v2:KHST_LEAF=v2" || exit 1
timeout -s KILL 150 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES SQ_INSTS_VMEM_RD --output-format csv -d gpurun_out/pmc_$tag -o pmc -- python3 bench.py --accounts 100000000 --steps 1 --warmup 1 --no-cpu > gpurun_out/pmc_$tag.log 2>&1
echo PMC_RC=$?
