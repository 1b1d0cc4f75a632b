# GEMM contention per tile shape on 8 concurrent CPX slices
set -u
mkdir -p gpurun_out/r2o
timeout -k 10 400 python tools/contention.py --mode cpx --ops qkv,fc2 --tiles 0,3,12,14,23,29,102,104 --out gpurun_out/r2o/tiles_cpx.json > gpurun_out/r2o/tiles_cpx.log 2>&1
