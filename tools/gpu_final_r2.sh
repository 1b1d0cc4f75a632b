# final-tree round: GPU suite, smoke, default bench, 200-quantum bench, sharing curve, rocprof kernel stats
set -u
mkdir -p gpurun_out/fin
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/fin/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/fin/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/fin/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/fin/smoke.log 2>&1 || { tail -30 gpurun_out/fin/smoke.log; exit 1; }
tail -1 gpurun_out/fin/smoke.log
timeout -k 10 300 python bench.py --out gpurun_out/fin/bench.json > gpurun_out/fin/bench.out 2> gpurun_out/fin/bench.err || { tail -20 gpurun_out/fin/bench.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/fin/bench.json')); print('bench', d['value'], d['inference_latency_ms'], d['pods_per_gpu_saturation'], d['density']['xcp'].get('inf_per_s_per_gpu'))"
timeout -k 10 600 python bench.py --steps 200 --warmup 5 --no-density --out gpurun_out/fin/bench200.json > /dev/null 2> gpurun_out/fin/bench200.err || { tail -20 gpurun_out/fin/bench200.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/fin/bench200.json')); print('bench200', d['value'], d['gpu_utilization_pct'], d['flips'], d['time_in_flip_pct'], d['hw_busy_pct'], d['inference_latency_ms'])"
timeout -k 10 500 python tools/sharing_curve.py --seconds 4 --out gpurun_out/fin/sharing_curve.json > gpurun_out/fin/curve.log 2>&1 || { tail -20 gpurun_out/fin/curve.log; exit 1; }
tail -6 gpurun_out/fin/curve.log
bash tools/gpu_prof_bench.sh
