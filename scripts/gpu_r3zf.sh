#!/bin/bash
# schedule A/B (scripts/gpu_sched_ab.sh), then the round-end evidence part A
export TMPDIR=/tmp
tag=${1:-r3e}
bash scripts/gpu_sched_ab.sh ${tag}s || exit $?
bash scripts/gpu_final_a.sh ${tag}
