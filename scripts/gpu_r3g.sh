#!/bin/bash
# round 3: parity (get, segmented 32-bit sort, sharded segmented C ABI, storage synth),
# sorted-leaf A/B, configs[3] sort A/B, the storage workload line
export TMPDIR=/tmp
tag=${1:-r3g}
step() { local name=$1; shift; "$@"; local rc=$?; echo "${name}_RC=$rc" >&2; [ $rc -eq 0 ] || exit $rc; }
step PYTEST timeout -k 10 700 python -u -m pytest tests/test_gpu_resident.py tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_sharded_cabi.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_$tag.log 2>&1
tail -1 gpurun_out/pytest_$tag.log
step STORAGE timeout -k 10 300 python bench.py --workload storage --steps 5 --warmup 2 > gpurun_out/storage_$tag.json 2> gpurun_out/storage_$tag.err
cut -c1-900 gpurun_out/storage_$tag.json
step SORTED env KHST_LEAF=sorted timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_${tag}_sorted.log 2>&1
tail -1 gpurun_out/pytest_${tag}_sorted.log
step AB bash scripts/gpu_ab_lib.sh $tag "input:X=1" "sorted:KHST_LEAF=sorted"
step CFG4CK timeout -k 10 300 python -u scripts/bench_configs.py --cfg 4 --no-cpu > gpurun_out/cfg4_${tag}_ck.json 2> gpurun_out/cfg4_${tag}_ck.err
step CFG4W64 env KHST_SEG_CK=0 timeout -k 10 300 python -u scripts/bench_configs.py --cfg 4 --no-cpu > gpurun_out/cfg4_${tag}_64.json 2> gpurun_out/cfg4_${tag}_64.err
for v in ck 64; do
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().split(chr(10))[-1]); print(sys.argv[1], round(d['ms'],2), {k: round(x,2) for k,x in d['stage_ms'].items()})" gpurun_out/cfg4_${tag}_$v.json
done
