set -u
mkdir -p gpurun_out/r2aj
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_kernels.py -k "fp32_input" > gpurun_out/r2aj/pytest.log 2>&1 || exit 1
NOS_ATTN_X3_FLAGS=2 timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_kernels.py -k "fp32_input" >> gpurun_out/r2aj/pytest.log 2>&1 || exit 1
for rep in 1 2; do for f in 0 2; do
  NOS_ATTN_X3_FLAGS=$f timeout -k 10 300 python tools/model_replay.py --slice spx --replays 40 >> gpurun_out/r2aj/replay_f$f.log 2>&1 || exit 1
done; done
for f in 0 2; do
  NOS_ATTN_X3_FLAGS=$f timeout -k 10 300 python tools/kbench.py --only modes --slices cpx,dpx --out gpurun_out/r2aj/modes_f$f.json > gpurun_out/r2aj/modes_f$f.log 2>&1 || exit 1
done
