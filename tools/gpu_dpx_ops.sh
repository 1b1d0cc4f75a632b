# per-op times on a 128-CU slice alone vs both halves busy (the request-lane layout), and the bench with latency
set -u
mkdir -p gpurun_out/dpx
timeout -k 10 400 python tools/contention.py --mode dpx --out gpurun_out/dpx/contention_dpx.json > gpurun_out/dpx/contention.log 2>&1 || { tail -20 gpurun_out/dpx/contention.log; exit 1; }
tail -12 gpurun_out/dpx/contention.log
timeout -k 10 300 python bench.py --no-density --out gpurun_out/dpx/bench.json > /dev/null 2> gpurun_out/dpx/bench.err || { tail -20 gpurun_out/dpx/bench.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/dpx/bench.json')); print('bench', d['value'], d['inference_latency_ms'])"
