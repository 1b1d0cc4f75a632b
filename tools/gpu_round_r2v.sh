set -u
mkdir -p gpurun_out/r2v
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r2v/pytest_gpu.log 2>&1 || exit 1
timeout -k 10 600 python bench.py > gpurun_out/r2v/bench.json 2> gpurun_out/r2v/bench.err || exit 1
