# box probe: does a persistent grid of exactly 256 workgroups straggle on this box? attention and
# persistent GEMM (fc1 tile 107) at full grid vs 4 short
set -u
mkdir -p gpurun_out/r2am
hostname > gpurun_out/r2am/host.txt 2>/dev/null || true
timeout -k 10 300 python tools/attn_grid.py --grids 256,252,248 --slices spx --out /tmp/x.json > gpurun_out/r2am/attn.log 2>&1 || exit 1
for sl in 0 4; do
  NOS_X3_PGRID_SLACK=$sl timeout -k 10 300 python tools/contention.py --mode spx --ops fc1,qkv --tiles 107,102 --out gpurun_out/r2am/g$sl.json > /dev/null 2>&1 || exit 1
done
