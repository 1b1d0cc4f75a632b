mkdir -p gpurun_out/r2k
timeout -k 10 300 python tools/operator_gpu_report.py --out gpurun_out/r2k/operator.json > gpurun_out/r2k/operator.log 2>&1 || exit 1
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/r2k_probe -o run -- python3 tools/clock_probe.py --out gpurun_out/r2k/clock.json > gpurun_out/r2k/clock_prof.log 2>&1 || exit 1
find /tmp/r2k_probe -name "*kernel_stats.csv" -exec cp {} gpurun_out/r2k/probe_kernel_stats.csv \;
