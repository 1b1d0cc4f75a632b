# smoke() and a 2-rank rehearsal of the multi-GPU bench (gloo, both ranks on the one GPU)
set -u
mkdir -p gpurun_out/s2
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/s2/smoke.log 2>&1 || { tail -30 gpurun_out/s2/smoke.log; exit 1; }
tail -1 gpurun_out/s2/smoke.log
NOS_BENCH_DIST_BACKEND=gloo timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 10 --warmup 2 --no-density > gpurun_out/s2/bench2.log 2>&1 || { tail -30 gpurun_out/s2/bench2.log; exit 1; }
grep metric gpurun_out/s2/bench2.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['n_gpus'], d['gpu_utilization_pct'], d['flips'], d['pods_per_node'])"
