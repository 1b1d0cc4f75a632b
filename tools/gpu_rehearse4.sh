# 4-rank rehearsal of the multi-GPU bench (gloo; all ranks share the one GPU of the box)
set -u
mkdir -p gpurun_out/r4
NOS_BENCH_DIST_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29541 bench.py --gpus 4 --steps 10 --warmup 2 > gpurun_out/r4/bench4.log 2>&1 || { tail -30 gpurun_out/r4/bench4.log; exit 1; }
grep metric gpurun_out/r4/bench4.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['n_gpus'], d['gpu_utilization_pct'], d['flips'], d['pods_per_node'], d['pods_per_gpu_saturation'], d['density']['xcp'])"
