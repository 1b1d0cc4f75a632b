# final-tree confirmation: GPU suite and two default bench runs (the driver's command)
set -u
mkdir -p gpurun_out/conf
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/conf/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/conf/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/conf/pytest_gpu.log
for r in 1 2; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --out gpurun_out/conf/bench_$r.json > /dev/null 2> gpurun_out/conf/bench_$r.err || { tail -20 gpurun_out/conf/bench_$r.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/conf/bench_$r.json')); print('bench', d['value'], d['ms_per_step'], d['hw_busy_pct'], d['inference_latency_ms'])"
done
