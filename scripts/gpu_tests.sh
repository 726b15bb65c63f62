#!/bin/bash
# GPU tests only (optionally a -k filter): python -u, per-test timeout, log under gpurun_out/
export TMPDIR=/tmp
TAG=${1:-t}
shift
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread -o log_cli=false "$@" > gpurun_out/pytest_$TAG.log 2>&1
rc=$?
tail -30 gpurun_out/pytest_$TAG.log
exit $rc
