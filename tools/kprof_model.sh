# rocprofv3 kernel stats of whole YOLOS-small inferences on one slice size (default SPX).
set -u
ROOT=$PWD
OUT=$ROOT/gpurun_out/mprof
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o model -- python3 $ROOT/tools/kbench.py --only model --slices ${1:-spx} --iters 8 --out $OUT/kb.json > $OUT/run.log 2>&1
rc=$?
tail -2 $OUT/run.log
exit $rc
