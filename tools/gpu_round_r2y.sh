set -u
mkdir -p gpurun_out/r2y
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_kernels.py -k "gemm_x3 or attention_x3" > gpurun_out/r2y/pytest.log 2>&1 || exit 1
NOS_X3_GROUP_M=4 timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_kernels.py -k "gemm_x3" > gpurun_out/r2y/pytest_g4.log 2>&1 || exit 1
timeout -k 10 300 python tools/attn_grid.py --grids 256,252,248 --slices spx,dpx --out gpurun_out/r2y/attn_grid.json > gpurun_out/r2y/attn_grid.log 2>&1 || exit 1
for g in 1 2 4 8; do
  NOS_X3_GROUP_M=$g timeout -k 10 300 python tools/contention.py --mode spx --ops qkv,proj,fc1,fc2 --out gpurun_out/r2y/spx_g$g.json > gpurun_out/r2y/spx_g$g.log 2>&1 || exit 1
done
