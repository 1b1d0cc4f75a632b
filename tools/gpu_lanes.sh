# GPU suite, default bench, and the bench with CU-split request lanes (each GPU step under its own limit)
set -u
mkdir -p gpurun_out/lanes
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/lanes/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/lanes/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/lanes/pytest_gpu.log
for lc in 0 128 64; do
  timeout -k 10 300 python bench.py --no-density --lane-cus $lc --out gpurun_out/lanes/bench_lc$lc.json \
    > /dev/null 2> gpurun_out/lanes/bench_lc$lc.err || { tail -30 gpurun_out/lanes/bench_lc$lc.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/lanes/bench_lc$lc.json')); print('lane_cus $lc', d['value'], d['gpu_utilization_pct'], d['pods_per_gpu'], d['hw_busy_pct'])"
done
timeout -k 10 400 python tools/kbench.py --only modes --emulation spread --out gpurun_out/lanes/modes.json > gpurun_out/lanes/modes.log 2>&1 || { tail -20 gpurun_out/lanes/modes.log; exit 1; }
grep mode gpurun_out/lanes/modes.log | python -c "import sys,json; [print(json.loads(l)['mode'], json.loads(l)['inf_per_s_per_gpu']) for l in sys.stdin]"
