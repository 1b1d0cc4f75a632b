set -u
mkdir -p gpurun_out/r2ab
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_kernels.py tests/test_infra.py -m gpu > gpurun_out/r2ab/pytest.log 2>&1 || exit 1
timeout -k 10 300 python tools/model_replay.py --slice spx --replays 40 > gpurun_out/r2ab/replay.log 2>&1 || exit 1
timeout -k 10 300 python tools/model_replay.py --slice spx --replays 40 >> gpurun_out/r2ab/replay.log 2>&1
