export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread -o log_cli=false > gpurun_out/pytest_r5l.log 2>&1 || { tail -30 gpurun_out/pytest_r5l.log; exit 1; }
tail -2 gpurun_out/pytest_r5l.log
bash scripts/gpu_ab_fetch.sh r5l tbl3= tbl2=khipu_amd/libkhst_tbl2.so pos=khipu_amd/libkhst_pos.so
