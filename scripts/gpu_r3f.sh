#!/bin/bash
# round 3: parity of batched get + the segmented 32-bit sort; A/B of sorted-order leaves;
# configs[3] with the segmented 32-bit sort against the 64-bit composite sort
export TMPDIR=/tmp
tag=${1:-r3f}
timeout -k 10 600 python -u -m pytest tests/test_gpu_resident.py tests/test_gpu_parity.py tests/test_gpu_configs.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_$tag.log 2>&1 || { tail -40 gpurun_out/pytest_$tag.log; exit 1; }
tail -1 gpurun_out/pytest_$tag.log
KHST_LEAF=sorted timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 120 --timeout-method thread -k "accounts or storage or genesis or full_size" > gpurun_out/pytest_${tag}_sorted.log 2>&1 || { tail -40 gpurun_out/pytest_${tag}_sorted.log; exit 1; }
tail -1 gpurun_out/pytest_${tag}_sorted.log
bash scripts/gpu_ab_lib.sh $tag "input:X=1" "sorted:KHST_LEAF=sorted" || exit 1
timeout -k 10 300 python -u scripts/bench_configs.py --cfg 4 --no-cpu > gpurun_out/cfg4_${tag}_ck.json 2>&1 || { tail gpurun_out/cfg4_${tag}_ck.json; exit 1; }
KHST_SEG_CK=0 timeout -k 10 300 python -u scripts/bench_configs.py --cfg 4 --no-cpu > gpurun_out/cfg4_${tag}_64.json 2>&1 || { tail gpurun_out/cfg4_${tag}_64.json; exit 1; }
for v in ck 64; do
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().split(chr(10))[-1]); print(sys.argv[1], round(d['ms'],2), {k: round(x,2) for k,x in d['stage_ms'].items()})" gpurun_out/cfg4_${tag}_$v.json
done
