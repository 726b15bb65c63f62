#!/bin/bash
# full GPU test suite, then the default 100M bench (no CPU legs) twice and a kernel profile
export TMPDIR=/tmp
tag=${1:-x}
timeout -k 10 800 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > gpurun_out/pytest_$tag.log 2>&1 || { tail -40 gpurun_out/pytest_$tag.log; exit 1; }
tail -1 gpurun_out/pytest_$tag.log
for r in 1 2; do
  timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu > gpurun_out/bench_${tag}_$r.json 2> gpurun_out/bench_${tag}_$r.err || { tail gpurun_out/bench_${tag}_$r.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/bench_${tag}_$r.json'));print(round(d['ms_per_step'],2), d['state_root'][:12], {k: round(v,2) for k,v in d['stage_ms'].items()})"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$tag -o prof -- python bench.py --steps 3 --warmup 1 --no-cpu > gpurun_out/prof_$tag.log 2>&1 || exit 1
python3 scripts/kstats.py gpurun_out/prof_$tag > gpurun_out/kstats_$tag.txt && head -16 gpurun_out/kstats_$tag.txt
