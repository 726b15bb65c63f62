#!/bin/bash
# PMC passes (each counter group in its own run, --kernel-trace only; MI355X_MICROARCH.md §rocprofv3).
export TMPDIR=/tmp
TAG=${1:-pmc}
N=${PMC_ACCOUNTS:-10000000}
rocprofv3 -L > gpurun_out/counters_list.txt 2>&1 || true
i=0
for PMC in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES" "GRBM_GUI_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAIT_INST_ANY"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $PMC --kernel-trace --output-format csv -d gpurun_out/${TAG}_p$i -o pmc -- python bench.py --accounts $N --steps 1 --warmup 1 --no-cpu > gpurun_out/${TAG}_p$i.log 2>&1
  rc=$?; echo "PMC pass $i ($PMC) rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 gpurun_out/${TAG}_p$i.log; exit $rc; fi
done
