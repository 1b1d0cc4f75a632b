# L2 behaviour of a partition mode with all of its partitions busy vs one alone (PMC pass with
# kernel trace only):   bash tools/pmc_modes.sh <mode> <partitions>
set -u
ROOT=$PWD
M=${1:-cpx}
N=${2:-8}
OUT=$ROOT/gpurun_out/pmc_modes_${M}_${N}
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TCC_EA0_RDREQ_sum --kernel-trace \
  --output-format csv -d $OUT -o p -- python3 $ROOT/tools/kbench.py --only modes --slices $M --partitions $N \
  --out $OUT/kb.json > $OUT/run.log 2>&1
rc=$?
tail -n 2 $OUT/run.log
exit $rc
