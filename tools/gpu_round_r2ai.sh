# fp32-input attention: numerics, then same-box A/B on whole inferences (SPX/DPX) and CPX 8-way
set -u
mkdir -p gpurun_out/r2ai
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_kernels.py -k "attention_x3 or yolos" > gpurun_out/r2ai/pytest.log 2>&1 || exit 1
for rep in 1 2; do for f in 0 1; do
  NOS_ATTN_F32IN=$f timeout -k 10 300 python tools/model_replay.py --slice spx --replays 40 >> gpurun_out/r2ai/replay_f$f.log 2>&1 || exit 1
  NOS_ATTN_F32IN=$f timeout -k 10 300 python tools/model_replay.py --slice dpx --replays 20 >> gpurun_out/r2ai/replay_f$f.log 2>&1 || exit 1
done; done
for f in 0 1; do
  NOS_ATTN_F32IN=$f timeout -k 10 300 python tools/kbench.py --only modes --slices cpx,qpx --out gpurun_out/r2ai/modes_f$f.json > gpurun_out/r2ai/modes_f$f.log 2>&1 || exit 1
done
