# the 10-s bench window across churn seeds on the final tree (the layout the window catches differs per seed)
set -u
mkdir -p gpurun_out/seeds
for seed in 1 2 3 4 5 1234; do
  timeout -k 10 300 python bench.py --no-density --seed $seed --out gpurun_out/seeds/b_$seed.json > /dev/null 2> gpurun_out/seeds/b_$seed.err || { tail -20 gpurun_out/seeds/b_$seed.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/seeds/b_$seed.json')); print('seed $seed', d['value'], d['gpu_utilization_pct'], d['flips'], list(d['inference_latency_ms']))"
done
