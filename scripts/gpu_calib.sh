#!/bin/bash
# FETCH_SIZE / WRITE_SIZE calibration (scripts/fetch_calib.hip), one PMC pass per counter.
export TMPDIR=/tmp
timeout -k 10 60 ./scripts/fetch_calib > gpurun_out/calib_known.txt || exit 1
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d gpurun_out/calib_rd -o c -- ./scripts/fetch_calib > gpurun_out/calib_rd.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d gpurun_out/calib_wr -o c -- ./scripts/fetch_calib > gpurun_out/calib_wr.log 2>&1 || exit 1
python scripts/fetch_calib.py gpurun_out/calib_rd gpurun_out/calib_wr gpurun_out/calib_known.txt --json gpurun_out/calib.json
