# PMC passes (counters in their own runs, kernel trace only) over one op on one slice:
#   bash tools/pmc_x3.sh <op> <slice>
set -u
ROOT=$PWD
OP=${1:-attn_x3}
SL=${2:-spx}
TILE=${3:-}
OUT=$ROOT/gpurun_out/pmc_${OP}_${SL}${TILE:+_t$TILE}
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
run() {  # run <tag> <counters...>
  local tag=$1; shift
  timeout -s KILL 90 rocprofv3 --pmc "$@" --kernel-trace --output-format csv -d $OUT -o $tag -- \
    python3 $ROOT/tools/kdrive.py --op $OP --slice $SL ${TILE:+--tile $TILE} > $OUT/$tag.log 2>&1
}
run p1 SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU && \
run p2 SQ_WAVES SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE GRBM_COUNT && \
run p3 TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum && \
run p4 SQ_INSTS_VMEM_RD SQ_INST_LEVEL_VMEM SQ_ACTIVE_INST_VMEM SQ_LDS_UNALIGNED_STALL SQ_LDS_ADDR_CONFLICT SQ_VALU_MFMA_COEXEC_CYCLES SQ_INST_CYCLES_VMEM_RD SQ_INSTS_LDS_STORE && \
run p5 TA_TA_BUSY_sum TA_BUFFER_READ_WAVEFRONTS_sum TD_TD_BUSY_sum GRBM_GUI_ACTIVE
rc=$?
for f in $OUT/*.log; do tail -n 2 "$f"; done
exit $rc
