# final-tree numbers: per-mode throughput (all partitions busy), the reference's sharing curve, a 200-quantum bench
set -u
mkdir -p gpurun_out/final
timeout -k 10 400 python tools/kbench.py --only modes --emulation spread --out gpurun_out/final/modes.json > gpurun_out/final/modes.log 2>&1 || { tail -20 gpurun_out/final/modes.log; exit 1; }
grep mode gpurun_out/final/modes.log | python -c "import sys,json; [print(json.loads(l)['mode'], json.loads(l)['inf_per_s_per_gpu']) for l in sys.stdin]"
timeout -k 10 500 python tools/sharing_curve.py --seconds 4 --out gpurun_out/final/sharing_curve.json > gpurun_out/final/curve.log 2>&1 || { tail -20 gpurun_out/final/curve.log; exit 1; }
tail -6 gpurun_out/final/curve.log
timeout -k 10 600 python bench.py --steps 200 --warmup 5 --no-density --out gpurun_out/final/bench200.json > /dev/null 2> gpurun_out/final/bench200.err || { tail -20 gpurun_out/final/bench200.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/final/bench200.json')); print('bench200', d['value'], d['gpu_utilization_pct'], d['flips'], d['time_in_flip_pct'], d['hw_busy_pct'])"
