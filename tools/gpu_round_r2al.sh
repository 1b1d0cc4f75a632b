# same-box A/B: stream-K XCD-major remap (flags 0) vs physical order (flags 4), grids 252/256 and 126/128
set -u
mkdir -p gpurun_out/r2al
timeout -k 10 300 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_kernels.py -k "attention_x3" > gpurun_out/r2al/pytest.log 2>&1 || exit 1
NOS_ATTN_X3_FLAGS=4 timeout -k 10 300 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_kernels.py -k "attention_x3" >> gpurun_out/r2al/pytest.log 2>&1 || exit 1
for rep in 1 2 3; do for f in 0 4; do
  NOS_ATTN_X3_FLAGS=$f timeout -k 10 300 python tools/attn_grid.py --grids 252,256 --slices spx --out /tmp/x.json >> gpurun_out/r2al/attn_f$f.log 2>&1 || exit 1
  NOS_ATTN_X3_FLAGS=$f timeout -k 10 300 python tools/attn_grid.py --grids 126,128 --slices dpx --out /tmp/x.json >> gpurun_out/r2al/attn_f$f.log 2>&1 || exit 1
done; done
for f in 0 4; do
  NOS_ATTN_X3_FLAGS=$f timeout -k 10 300 python tools/model_replay.py --slice spx --replays 40 >> gpurun_out/r2al/replay_f$f.log 2>&1 || exit 1
done
