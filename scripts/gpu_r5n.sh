export TMPDIR=/tmp
timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/smoke_r5n.log 2>&1 || { tail -20 gpurun_out/smoke_r5n.log; exit 1; }
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread -o log_cli=false > gpurun_out/pytest_r5n.log 2>&1 || { tail -30 gpurun_out/pytest_r5n.log; exit 1; }
tail -2 gpurun_out/pytest_r5n.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r5n -o prof -- python3 bench.py --steps 3 --warmup 1 --no-cpu --no-host-path > gpurun_out/prof_r5n.log 2>&1 || exit 1
for r in 1 2; do timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu --no-host-path > gpurun_out/bench_r5n_$r.json 2>/dev/null || exit 1; python -c "import json;d=json.load(open('gpurun_out/bench_r5n_$r.json'));print(round(d['ms_per_step'],2), {k: round(v,2) for k,v in d['stage_ms'].items()})"; done
