export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread -o log_cli=false > gpurun_out/pytest_r5o.log 2>&1 || { tail -30 gpurun_out/pytest_r5o.log; exit 1; }
tail -2 gpurun_out/pytest_r5o.log
bash scripts/gpu_block_trace.sh r5o || exit 1
timeout -k 10 600 python scripts/bench_configs.py --cfg 3 --no-cpu --steps 10 --warmup 3 > gpurun_out/cfg3_r5o.json 2> gpurun_out/cfg3_r5o.err || { tail -5 gpurun_out/cfg3_r5o.err; exit 1; }; python -c "import json;d=json.load(open(\"gpurun_out/cfg3_r5o.json\"));print(d[\"block_ms_median\"], d[\"block_ms_all\"])"
