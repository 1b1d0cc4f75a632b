# LDS / MFMA counters of the QKV x3 GEMM on a 128-CU slice: 128x128 tiles (64x32 waves: 14, 29) vs
# the 256x128 8-wave tiles (64x64 waves: 35, 36), one tile per pass
set -u
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/pmc_t256
mkdir -p $OUT
cd /tmp
for tile in 14 29 35 36; do
  timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES SQ_WAVE_CYCLES SQ_INSTS_MFMA --kernel-trace -d $OUT/qkv_$tile -o p --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/kdrive.py --op qkv_x3 --slice dpx --tile $tile --iters 5 > $OUT/qkv_$tile.log 2>&1 || { tail -20 $OUT/qkv_$tile.log; exit 1; }
  echo "qkv $tile ok"
done
cd $GRAFT_REPO_ROOT && python3 tools/pmc_summary.py gpurun_out/pmc_t256/qkv_14 gpurun_out/pmc_t256/qkv_29 gpurun_out/pmc_t256/qkv_35 gpurun_out/pmc_t256/qkv_36 > gpurun_out/pmc_t256/summary.txt && cat gpurun_out/pmc_t256/summary.txt
