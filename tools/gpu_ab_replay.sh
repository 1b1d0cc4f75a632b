# same-box A/B of one whole-GPU inference (graph replay): ENV=value pairs given as arguments, each
# run twice in alternation; e.g. bash tools/gpu_ab_replay.sh NOS_SPLITK=0 NOS_SPLITK=1
set -u
mkdir -p gpurun_out/ab
for rep in 1 2; do
  for kv in "$@"; do
    env "$kv" timeout -k 10 300 python tools/model_replay.py --slice spx --replays 100 > gpurun_out/ab/replay.log 2>&1 || { tail -20 gpurun_out/ab/replay.log; exit 1; }
    echo "$kv $(tail -1 gpurun_out/ab/replay.log)"
  done
done
