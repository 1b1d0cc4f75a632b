mkdir -p gpurun_out
timeout -k 10 300 python tools/kbench.py --only modes --out gpurun_out/r2i_modes.json > gpurun_out/r2i_modes.log 2>&1 || exit 1
NOS_BENCH_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 8 --warmup 2 --preroll 20 --no-density > gpurun_out/r2i_bench_2rank.log 2>&1 || exit 1
timeout -k 10 400 python bench.py --out gpurun_out/r2i_bench.json > gpurun_out/r2i_bench.log 2>&1
