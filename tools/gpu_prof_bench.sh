# rocprofv3 kernel trace + stats of the default bench on the current tree; window summary of the timed steps
set -u
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/profb
mkdir -p $OUT
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT -o bench --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --no-density > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
python3 $GRAFT_REPO_ROOT/tools/trace_window.py $OUT/bench_kernel_trace.csv --tail-frac 0.4 > $OUT/window.txt
head -14 $OUT/window.txt; rm -f $OUT/bench_kernel_trace.csv
grep -o '"value": [0-9.]*' $OUT/bench.json
