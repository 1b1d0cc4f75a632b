# contention vs the HIP runtime's hardware-queue count (8 CU-masked streams; default is 4 queues)
set -u
mkdir -p gpurun_out/r2n
for q in 8 16; do
  GPU_MAX_HW_QUEUES=$q timeout -k 10 300 python tools/contention.py --mode cpx --head-blocks 6 --out gpurun_out/r2n/contention_cpx_q$q.json > gpurun_out/r2n/contention_cpx_q$q.log 2>&1 || exit 1
done
GPU_MAX_HW_QUEUES=8 timeout -k 10 300 python tools/kbench.py --only modes --out gpurun_out/r2n/modes_q8.json > gpurun_out/r2n/modes_q8.log 2>&1
