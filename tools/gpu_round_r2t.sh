set -u
mkdir -p gpurun_out/r2t
timeout -k 10 300 python tools/attn_grid.py --grids 256,255,254,252,250,248,244,236,224 --slices spx --out gpurun_out/r2t/spx.json > gpurun_out/r2t/spx.log 2>&1 || exit 1
timeout -k 10 300 python tools/attn_grid.py --grids 64,63,62,60,56 --slices qpx --out gpurun_out/r2t/qpx.json > gpurun_out/r2t/qpx.log 2>&1 || exit 1
timeout -k 10 300 python tools/attn_grid.py --grids 32,31,30,28 --slices cpx --out gpurun_out/r2t/cpx.json > gpurun_out/r2t/cpx.log 2>&1
