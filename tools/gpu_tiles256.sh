# 256x128 / 128x256 8-wave x3 GEMM tiles: numerics on every shape, then alone/concurrent timings vs the current tiles
set -u
mkdir -p gpurun_out/t256
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 300 --timeout-method thread -k "gemm_x3_every_tile or splitk" \
  > gpurun_out/t256/pytest.log 2>&1 || { tail -30 gpurun_out/t256/pytest.log; exit 1; }
tail -2 gpurun_out/t256/pytest.log
for mode in dpx qpx; do
  timeout -k 10 300 python tools/contention.py --mode $mode --ops qkv_f32,qkv --tiles 14,29,35,36 --out gpurun_out/t256/qkv_$mode.json > gpurun_out/t256/qkv_$mode.log 2>&1 || { tail -20 gpurun_out/t256/qkv_$mode.log; exit 1; }
  grep op gpurun_out/t256/qkv_$mode.log
  timeout -k 10 300 python tools/contention.py --mode $mode --ops fc1,fc1_f32 --tiles 14,29,35,36,37 --out gpurun_out/t256/fc1_$mode.json > gpurun_out/t256/fc1_$mode.log 2>&1 || { tail -20 gpurun_out/t256/fc1_$mode.log; exit 1; }
  grep op gpurun_out/t256/fc1_$mode.log
done
