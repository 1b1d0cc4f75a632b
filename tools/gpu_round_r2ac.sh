# reference demo reproduction (1/3/5/7 pods, three sharing modes) + 2-rank multi-process bench rehearsal
set -u
mkdir -p gpurun_out/r2ac
timeout -k 10 600 python tools/sharing_curve.py --seconds 5 --out gpurun_out/r2ac/sharing_curve.json > gpurun_out/r2ac/sharing_curve.log 2>&1 || exit 1
NOS_BENCH_DIST_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 10 --warmup 2 --no-density > gpurun_out/r2ac/bench_2rank_gloo.log 2>&1
