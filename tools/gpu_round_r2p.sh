# grid-stride LayerNorm + persistent x3 GEMM tiles under 8/4 concurrent slices
set -u
mkdir -p gpurun_out/r2p
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "layernorm or attention_x3" > gpurun_out/r2p/pytest.log 2>&1 || exit 1
timeout -k 10 300 python tools/contention.py --mode cpx --ops ln --out gpurun_out/r2p/ln_cpx.json > gpurun_out/r2p/ln_cpx.log 2>&1 || exit 1
timeout -k 10 400 python tools/contention.py --mode cpx --ops qkv,proj,fc1,fc2 --tiles 14,29,100,101,102,103,104,105,107,108,109 --out gpurun_out/r2p/tiles_cpx.json > gpurun_out/r2p/tiles_cpx.log 2>&1 || exit 1
timeout -k 10 400 python tools/contention.py --mode qpx --ops qkv,proj,fc1,fc2 --tiles 14,29,100,101,102,103,104,105,107,108,109 --out gpurun_out/r2p/tiles_qpx.json > gpurun_out/r2p/tiles_qpx.log 2>&1
