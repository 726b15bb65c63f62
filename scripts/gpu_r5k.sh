export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread -o log_cli=false > gpurun_out/pytest_r5k.log 2>&1 || { tail -30 gpurun_out/pytest_r5k.log; exit 1; }
tail -2 gpurun_out/pytest_r5k.log
bash scripts/gpu_ab_fetch.sh r5k tbl= pos=khipu_amd/libkhst_pos.so w3=khipu_amd/libkhst_w3.so w2=khipu_amd/libkhst_w2.so pdf=khipu_amd/libkhst_pdf.so
