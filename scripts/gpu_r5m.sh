export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread -o log_cli=false > gpurun_out/pytest_r5m.log 2>&1 || { tail -30 gpurun_out/pytest_r5m.log; exit 1; }
tail -2 gpurun_out/pytest_r5m.log
bash scripts/gpu_ab_fetch.sh r5m k1tbl= k1pos=khipu_amd/libkhst_k1pos.so pos=khipu_amd/libkhst_pos.so || exit 1
bash scripts/gpu_block_trace.sh r5m
