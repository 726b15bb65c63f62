#!/bin/bash
# Branch levels at fewer waves per CU (KHST_BR_LDS_PAD: extra LDS per 256-thread block of
# k_branch_fused; 35 KB static -> 4 blocks per CU; +6 KB -> 3; +20 KB -> 2): 100M step A/B
export TMPDIR=/tmp
step() { local name=$1; shift; "$@"; local rc=$?; echo "${name}_RC=$rc" >&2; [ $rc -eq 0 ] || exit $rc; }
step AB bash scripts/gpu_ab_lib.sh r4ba "p0:X=1" "p6k:KHST_BR_LDS_PAD=6144" "p20k:KHST_BR_LDS_PAD=20480"
echo done
