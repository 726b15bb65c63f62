export TMPDIR=/tmp
set -o pipefail
timeout -k 10 300 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread -k "variants or genesis or full_size" > gpurun_out/pytest_r2c.log 2>&1 && tail -2 gpurun_out/pytest_r2c.log && \
KHST_BRANCH=coop timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu > gpurun_out/bench_r2c_coop.json 2>/dev/null && \
KHST_BRANCH=lane timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu > gpurun_out/bench_r2c_lane.json 2>/dev/null && \
KHST_BRANCH=coop timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r2c -o prof -- python bench.py --steps 2 --warmup 1 --no-cpu > gpurun_out/prof_r2c.log 2>&1 && \
python scripts/kstats.py gpurun_out/prof_r2c > gpurun_out/kstats_r2c.txt && head -12 gpurun_out/kstats_r2c.txt
