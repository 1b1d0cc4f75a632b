set -u
ROOT=$PWD
mkdir -p gpurun_out/kprof
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $ROOT/gpurun_out/kprof -o kb --output-format csv -- python3 $ROOT/tools/kbench.py --only attn --slices spx,dpx,cpx --iters 10 --out $ROOT/gpurun_out/kbench_attn.json > $ROOT/gpurun_out/kprof.log 2>&1
rc=$?
tail -5 $ROOT/gpurun_out/kprof.log
exit $rc
