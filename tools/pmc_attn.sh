# PMC counters for the attention and GEMM kernels on SPX and CPX slices (counters in their own run,
# kernel trace only; see cdna_hip_programming.md §7).
set -u
ROOT=$PWD
OUT=$ROOT/gpurun_out/pmc
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
timeout -k 10 60 rocprofv3 -L > $OUT/counters.txt 2>&1 || true
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES GRBM_GUI_ACTIVE \
  --kernel-trace --output-format csv -d $OUT -o attn -- python3 $ROOT/tools/kbench.py --only ${1:-attn} --slices spx,cpx --iters 3 --out $OUT/kb.json > $OUT/run.log 2>&1
rc=$?
tail -3 $OUT/run.log
exit $rc
