set -u
mkdir -p gpurun_out/r2s
timeout -k 10 300 python tools/attn_grid.py --grids 256,252,240,224,192,168,128,84 --slices spx --out gpurun_out/r2s/attn_grid_spx.json > gpurun_out/r2s/attn_grid_spx.log 2>&1 || exit 1
timeout -k 10 300 python tools/attn_grid.py --grids 128,126,112,96,84 --slices dpx --out gpurun_out/r2s/attn_grid_dpx.json > gpurun_out/r2s/attn_grid_dpx.log 2>&1
