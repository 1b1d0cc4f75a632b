# same-box A/B of the x3 GEMM shapes and of one whole inference: ENV=value pairs as arguments
set -u
mkdir -p gpurun_out/abs
for kv in "$@"; do
  env "$kv" timeout -k 10 300 python tools/x3_shapes.py --out gpurun_out/abs/shapes_${kv}.json > gpurun_out/abs/shapes.log 2>&1 || { tail -20 gpurun_out/abs/shapes.log; exit 1; }
  echo "$kv"; cat gpurun_out/abs/shapes.log | grep -v amdgpu.ids
done
for rep in 1 2; do
  for kv in "$@"; do
    env "$kv" timeout -k 10 300 python tools/model_replay.py --slice spx --replays 100 > gpurun_out/abs/replay.log 2>&1 || { tail -20 gpurun_out/abs/replay.log; exit 1; }
    echo "$kv $(tail -1 gpurun_out/abs/replay.log)"
  done
done
