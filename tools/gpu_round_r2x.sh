# L2 / fabric counters per kernel of steady-state SPX inferences (PMC serialises dispatches: one stream anyway)
set -u
mkdir -p gpurun_out/r2x
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TCC_EA0_RDREQ_sum --kernel-trace --output-format csv -d /tmp/r2x/p1 -o p1 -- python3 tools/model_replay.py --slice spx --replays 4 > gpurun_out/r2x/p1.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d /tmp/r2x/p2 -o p2 -- python3 tools/model_replay.py --slice spx --replays 4 > gpurun_out/r2x/p2.log 2>&1 || exit 1
for p in p1 p2; do find /tmp/r2x/$p -name "*counter_collection.csv" -exec gzip -c {} \; > gpurun_out/r2x/${p}_counters.csv.gz; done
