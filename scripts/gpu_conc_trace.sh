export TMPDIR=/tmp
for mode in host device; do
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/conc_$mode -o ct -- python3 scripts/concurrency_probe.py $mode 1000000 12 > gpurun_out/conc_$mode.log 2>&1 || { tail -5 gpurun_out/conc_$mode.log; exit 1; }
grep throughput gpurun_out/conc_$mode.log
python scripts/conc_trace.py gpurun_out/conc_$mode --tail-ms 25 > gpurun_out/conc_${mode}_summary.json && cat gpurun_out/conc_${mode}_summary.json
done
