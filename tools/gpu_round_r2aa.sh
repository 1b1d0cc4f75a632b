set -u
mkdir -p gpurun_out/r2aa
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_kernels.py -k "attention_x3" > gpurun_out/r2aa/pytest.log 2>&1 || exit 1
for rep in 1 2; do for f in 0 1; do
  NOS_ATTN_X3_FLAGS=$f timeout -k 10 300 python tools/attn_grid.py --grids 256,252 --slices spx --out gpurun_out/r2aa/spx_f$f.json >> gpurun_out/r2aa/attn_f$f.log 2>&1 || exit 1
  NOS_ATTN_X3_FLAGS=$f timeout -k 10 300 python tools/attn_grid.py --grids 128,126 --slices dpx --out gpurun_out/r2aa/dpx_f$f.json >> gpurun_out/r2aa/attn_f$f.log 2>&1 || exit 1
  NOS_ATTN_X3_FLAGS=$f timeout -k 10 300 python tools/attn_grid.py --grids 32 --slices cpx --out gpurun_out/r2aa/cpx_f$f.json >> gpurun_out/r2aa/attn_f$f.log 2>&1 || exit 1
done; done
