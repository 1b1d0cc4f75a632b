# GPU suite + default bench on the current tree (each GPU step under its own limit; stop on failure)
set -u
mkdir -p gpurun_out/check
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/check/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/check/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/check/pytest_gpu.log
timeout -k 10 600 python bench.py > gpurun_out/check/bench.json 2> gpurun_out/check/bench.err || { tail -30 gpurun_out/check/bench.err; exit 1; }
cat gpurun_out/check/bench.json
