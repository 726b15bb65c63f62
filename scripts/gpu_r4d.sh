#!/bin/bash
# Round 4: the full GPU suite at HEAD, then configs[2] (50M resident, block commits) with and
# without kh_block_commit's journal (measurement build khipu_amd/libkhst_notxn.so).
export TMPDIR=/tmp
TAG=${1:-r4d}
step() { local name=$1; shift; "$@"; local rc=$?; echo "${name}_RC=$rc" >&2; [ $rc -eq 0 ] || exit $rc; }
step PYTEST timeout -k 10 1000 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread -o log_cli=false > gpurun_out/pytest_$TAG.log 2>&1
tail -3 gpurun_out/pytest_$TAG.log
for rep in 1 2; do
  step CFG3_TXN timeout -k 10 300 python scripts/bench_configs.py --cfg 3 --no-cpu > gpurun_out/cfg3_${TAG}_txn_$rep.jsonl 2> gpurun_out/cfg3_${TAG}_txn_$rep.err
  cut -c1-400 gpurun_out/cfg3_${TAG}_txn_$rep.jsonl
  step CFG3_NOTXN timeout -k 10 300 env KHST_LIB_AB=khipu_amd/libkhst_notxn.so python scripts/bench_configs.py --cfg 3 --no-cpu > gpurun_out/cfg3_${TAG}_notxn_$rep.jsonl 2> gpurun_out/cfg3_${TAG}_notxn_$rep.err
  cut -c1-400 gpurun_out/cfg3_${TAG}_notxn_$rep.jsonl
done
