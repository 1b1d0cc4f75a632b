# rocprofv3 kernel stats of CPX partitions: one busy slice vs all eight busy (contention diagnosis)
mkdir -p gpurun_out/r2j
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/r2j_one -o run -- python3 tools/kbench.py --only modes --slices cpx --partitions 1 --out gpurun_out/r2j/one.json > gpurun_out/r2j/one.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/r2j_eight -o run -- python3 tools/kbench.py --only modes --slices cpx --out gpurun_out/r2j/eight.json > gpurun_out/r2j/eight.log 2>&1 || exit 1
find /tmp/r2j_one -name "*kernel_stats.csv" -exec cp {} gpurun_out/r2j/one_kernel_stats.csv \;
find /tmp/r2j_eight -name "*kernel_stats.csv" -exec cp {} gpurun_out/r2j/eight_kernel_stats.csv \;
