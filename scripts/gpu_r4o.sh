#!/bin/bash
# Round 4: issue / wait breakdown of k_topo_tile (scatter as its own kernel: KHST_TOPO_TILE=2),
# serialized kernels, one PMC pass of SQ counters
export TMPDIR=/tmp
TAG=${1:-r4o}
export AMD_SERIALIZE_KERNEL=3 KHST_TOPO_TILE=2
timeout -s KILL 240 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/${TAG}_p1 -o pmc -- python3 bench.py --steps 1 --warmup 1 --no-cpu --no-host-path > gpurun_out/${TAG}_p1.log 2>&1
rc=$?; echo "PMC_RC=$rc"; [ $rc -eq 0 ] || exit $rc
python3 scripts/issue_summary.py gpurun_out/${TAG}_p1 > gpurun_out/${TAG}_issue.json && grep -A14 '"k_topo_tile"\|"k_pd_scatter"\|"k_branch_topo"' gpurun_out/${TAG}_issue.json
