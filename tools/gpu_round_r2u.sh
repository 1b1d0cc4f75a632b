set -u
mkdir -p gpurun_out/r2u
timeout -k 10 300 python tools/kbench.py --only model --slices spx,dpx --iters 8 --out gpurun_out/r2u/model.json > gpurun_out/r2u/model.log 2>&1 || exit 1
for sl in 0 4 8; do
  NOS_X3_PGRID_SLACK=$sl timeout -k 10 300 python tools/contention.py --mode spx --ops qkv,proj,fc1,fc2 --tiles 100,102,104,105,107,108,109 --out gpurun_out/r2u/pslack$sl.json > gpurun_out/r2u/pslack$sl.log 2>&1 || exit 1
done
