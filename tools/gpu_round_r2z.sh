set -u
mkdir -p gpurun_out/r2z
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_kernels.py -k "attention_x3" > gpurun_out/r2z/pytest.log 2>&1 || exit 1
timeout -k 10 300 python tools/attn_grid.py --grids 252 --slices spx --out gpurun_out/r2z/spx.json > gpurun_out/r2z/attn.log 2>&1 || exit 1
timeout -k 10 300 python tools/attn_grid.py --grids 126 --slices dpx --out gpurun_out/r2z/dpx.json >> gpurun_out/r2z/attn.log 2>&1 || exit 1
timeout -k 10 300 python tools/attn_grid.py --grids 64 --slices qpx --out gpurun_out/r2z/qpx.json >> gpurun_out/r2z/attn.log 2>&1 || exit 1
timeout -k 10 300 python tools/attn_grid.py --grids 32 --slices cpx --out gpurun_out/r2z/cpx.json >> gpurun_out/r2z/attn.log 2>&1
