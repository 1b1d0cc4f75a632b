# fused heads / patch planes: kernel tests, then one-inference replay time and its kernel trace
set -u
mkdir -p gpurun_out/head
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_pin.py -x -q --timeout 240 --timeout-method thread > gpurun_out/head/pytest.log 2>&1 || { tail -40 gpurun_out/head/pytest.log; exit 1; }
tail -2 gpurun_out/head/pytest.log
timeout -k 10 300 python tools/model_replay.py --slice spx --replays 40 > gpurun_out/head/replay.log 2>&1 || { tail -20 gpurun_out/head/replay.log; exit 1; }
tail -3 gpurun_out/head/replay.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/head/prof -o replay --output-format csv -- python3 tools/model_replay.py --slice spx --replays 40 > gpurun_out/head/prof.log 2>&1 || { tail -20 gpurun_out/head/prof.log; exit 1; }
find gpurun_out/head/prof -name "*kernel_stats.csv"
