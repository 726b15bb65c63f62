#!/bin/bash
# Keccak unroll, one box: HEAD (8 everywhere), hybrid (24 in key hashing and the leaf kernel, the
# working tree), 24 everywhere (-DKECCAK_LOOP_ROUNDS=24); 100M step, 3 rounds
export TMPDIR=/tmp
step() { local name=$1; shift; "$@"; local rc=$?; echo "${name}_RC=$rc" >&2; [ $rc -eq 0 ] || exit $rc; }
step AB bash scripts/gpu_ab_lib.sh r4bp "base:KHST_LIB_AB=khipu_amd/libkhst_base.so" "hyb:X=1" "u24:KHST_LIB_AB=khipu_amd/libkhst_u24.so"
step AB2 bash scripts/gpu_ab_lib.sh r4bp2 "u24:KHST_LIB_AB=khipu_amd/libkhst_u24.so" "hyb:X=1" "base:KHST_LIB_AB=khipu_amd/libkhst_base.so"
echo done
