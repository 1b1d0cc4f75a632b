# after the 256-wide tiles + re-measured table: GPU suite, per-mode throughput, default bench
set -u
mkdir -p gpurun_out/after
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/after/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/after/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/after/pytest_gpu.log
timeout -k 10 400 python tools/kbench.py --only modes --emulation spread --out gpurun_out/after/modes.json > gpurun_out/after/modes.log 2>&1 || { tail -20 gpurun_out/after/modes.log; exit 1; }
grep mode gpurun_out/after/modes.log | python -c "import sys,json; [print(json.loads(l)['mode'], json.loads(l)['inf_per_s_per_gpu']) for l in sys.stdin]"
timeout -k 10 300 python bench.py --out gpurun_out/after/bench.json > /dev/null 2> gpurun_out/after/bench.err || { tail -20 gpurun_out/after/bench.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/after/bench.json')); print('bench', d['value'], d['inference_latency_ms'], d['density']['xcp'])"
