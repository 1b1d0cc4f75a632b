# LDS / MFMA counters of the x3 GEMM tiles the tuner picks at SPX (fc1: r 64x128 and DMA 64x64 m16;
# qkv: DMA 128x128 m16 and 32x32; fc2: DMA 64x128 64-deep), one op per pass
set -u
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/pmc_lds
mkdir -p $OUT
cd /tmp
for spec in "fc1_x3 6" "fc1_x3 27" "qkv_x3 29" "qkv_x3 14" "fc2_x3 24" "attn_x3 -1"; do
  set -- $spec
  op=$1; tile=$2
  targ=""; [ "$tile" != "-1" ] && targ="--tile $tile"
  timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES SQ_WAVE_CYCLES SQ_INSTS_MFMA --kernel-trace -d $OUT/${op}_$tile -o p --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/kdrive.py --op $op --slice spx $targ --iters 5 > $OUT/${op}_$tile.log 2>&1 || { tail -20 $OUT/${op}_$tile.log; exit 1; }
  echo "$op $tile ok"
done
