# head-block attention: correctness, then per-op contention of concurrent CPX / QPX slices
set -u
mkdir -p gpurun_out/r2m
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "attention_x3" > gpurun_out/r2m/pytest.log 2>&1 || exit 1
timeout -k 10 300 python tools/contention.py --mode cpx --out gpurun_out/r2m/contention_cpx.json > gpurun_out/r2m/contention_cpx.log 2>&1 || exit 1
timeout -k 10 300 python tools/contention.py --mode qpx --out gpurun_out/r2m/contention_qpx.json > gpurun_out/r2m/contention_qpx.log 2>&1 || exit 1
timeout -k 10 300 python tools/contention.py --mode spx --ops attn --out gpurun_out/r2m/contention_spx.json > gpurun_out/r2m/contention_spx.log 2>&1
