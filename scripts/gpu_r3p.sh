#!/bin/bash
# round 3: issue / wait breakdown of the leaf kernel against key hashing, serialized kernels
# (one PMC pass of SQ counters; GRBM_GUI_ACTIVE for the effective clock)
export TMPDIR=/tmp
TAG=${1:-r3p}
export AMD_SERIALIZE_KERNEL=3
timeout -s KILL 240 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/${TAG}_p1 -o pmc -- python3 bench.py --steps 1 --warmup 1 --no-cpu > gpurun_out/${TAG}_p1.log 2>&1
rc=$?; echo "PMC_RC=$rc"; [ $rc -eq 0 ] || exit $rc
python3 scripts/issue_summary.py gpurun_out/${TAG}_p1 > gpurun_out/${TAG}_issue.json && cat gpurun_out/${TAG}_issue.json
