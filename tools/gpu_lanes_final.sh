# smoke(), a 2-rank rehearsal (gloo, both ranks on the one GPU) and a 200-quantum bench on the lanes default
set -u
bash tools/gpu_smoke_2rank.sh || exit 1
mkdir -p gpurun_out/final
timeout -k 10 600 python bench.py --steps 200 --warmup 5 --no-density --out gpurun_out/final/bench200.json > /dev/null 2> gpurun_out/final/bench200.err || { tail -20 gpurun_out/final/bench200.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/final/bench200.json')); print('bench200', d['value'], d['gpu_utilization_pct'], d['flips'], d['time_in_flip_pct'], d['hw_busy_pct'], d['pods_per_gpu'])"
