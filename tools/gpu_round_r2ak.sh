set -u
mkdir -p gpurun_out/r2ak
timeout -k 10 300 python tools/attn_grid.py --grids 252,256 --slices spx --out gpurun_out/r2ak/g8.json > gpurun_out/r2ak/log 2>&1 || exit 1
NOS_ATTN_X3_GROUP=4 timeout -k 10 300 python tools/attn_grid.py --grids 486,512,504,324 --slices spx --out gpurun_out/r2ak/g4.json >> gpurun_out/r2ak/log 2>&1 || exit 1
NOS_ATTN_X3_GROUP=4 timeout -k 10 300 python tools/attn_grid.py --grids 243,256,252,162 --slices dpx --out gpurun_out/r2ak/g4d.json >> gpurun_out/r2ak/log 2>&1 || exit 1
timeout -k 10 300 python tools/attn_grid.py --grids 126,128 --slices dpx --out gpurun_out/r2ak/g8d.json >> gpurun_out/r2ak/log 2>&1
