#!/bin/bash
# Round 4: block-commit tests, then configs[2] (50M resident) with the overlapped phases (default)
# and one after the other (measurement build khipu_amd/libkhst_serial.so), then the verify
# workload and the host-path bench.
export TMPDIR=/tmp
TAG=${1:-r4f}
step() { local name=$1; shift; "$@"; local rc=$?; echo "${name}_RC=$rc" >&2; [ $rc -eq 0 ] || exit $rc; }
step PYTEST timeout -k 10 900 python -u -m pytest tests/test_gpu_versioned.py tests/test_gpu_resident.py tests/test_gpu_configs.py -x -v -m gpu --timeout 300 --timeout-method thread -o log_cli=false > gpurun_out/pytest_$TAG.log 2>&1
tail -3 gpurun_out/pytest_$TAG.log
for rep in 1 2; do
  step CFG3 timeout -k 10 300 python scripts/bench_configs.py --cfg 3 --no-cpu > gpurun_out/cfg3_${TAG}_overlap_$rep.jsonl 2> gpurun_out/cfg3_${TAG}_overlap_$rep.err
  python -c "import json,sys;d=json.loads(open(sys.argv[1]).readline());print('overlap',round(d['block_ms_median'],3))" gpurun_out/cfg3_${TAG}_overlap_$rep.jsonl
  step CFG3S timeout -k 10 300 env KHST_LIB_AB=khipu_amd/libkhst_serial.so python scripts/bench_configs.py --cfg 3 --no-cpu > gpurun_out/cfg3_${TAG}_serial_$rep.jsonl 2> gpurun_out/cfg3_${TAG}_serial_$rep.err
  python -c "import json,sys;d=json.loads(open(sys.argv[1]).readline());print('serial',round(d['block_ms_median'],3))" gpurun_out/cfg3_${TAG}_serial_$rep.jsonl
done
bash scripts/gpu_r4e.sh $TAG
