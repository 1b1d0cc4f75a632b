set -u
mkdir -p gpurun_out/r2w
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/r2w -o m -- python3 tools/model_replay.py --slice spx --replays 40 > gpurun_out/r2w/run.log 2>&1 || exit 1
f=$(find /tmp/r2w -name "*kernel_trace.csv" | head -1)
python3 tools/trace_window.py "$f" --tail-frac 0.3 > gpurun_out/r2w/window.txt 2>&1
cp "$f" /tmp/kt.csv && gzip -c /tmp/kt.csv > gpurun_out/r2w/kernel_trace.csv.gz
