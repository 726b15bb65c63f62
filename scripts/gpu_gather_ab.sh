#!/bin/bash
# Block-commit gather A/B: the whole GPU suite on the new gather (records' pairs listed in
# LDS), then configs[2] at 50M alternating the default with KHST_GATHER=nibble (the
# previous one-thread-per-(record, nibble) form), and the block-commit kernel trace
export TMPDIR=/tmp
tag=${1:-ga}
step() { local name=$1; shift; "$@"; local rc=$?; echo "${name}_RC=$rc" >&2; [ $rc -eq 0 ] || exit $rc; }
step PYTEST timeout -k 10 700 python -u -m pytest tests -x -v -m gpu --timeout 200 --timeout-method thread -o log_cli=false > gpurun_out/pytest_$tag.log 2>&1
tail -2 gpurun_out/pytest_$tag.log
for v in def nib def2 nib2; do
  case $v in
    def*) envs="KHST_GATHER=pairs" ;;
    nib*) envs="KHST_GATHER=nibble" ;;
  esac
  step CFG2_$v env $envs timeout -k 10 400 python scripts/bench_configs.py --cfg 3 --no-cpu > gpurun_out/cfg2_${tag}_$v.jsonl 2> gpurun_out/cfg2_${tag}_$v.err
  cut -c1-330 gpurun_out/cfg2_${tag}_$v.jsonl
done
step BC timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/bc_$tag -o bc -- python3 scripts/block_commit_prof.py > gpurun_out/bc_$tag.log 2>&1
python3 scripts/block_trace.py gpurun_out/bc_$tag --timeline gpurun_out/bc_timeline_$tag.json > gpurun_out/bc_trace_$tag.json && head -c 1500 gpurun_out/bc_trace_$tag.json
