# bench with 1 vs 2 concurrent request streams per pod (same seed / window)
set -u
mkdir -p gpurun_out/streams
for k in 1 2; do
  timeout -k 10 400 python bench.py --pod-streams $k --no-density > gpurun_out/streams/bench_s$k.json 2> gpurun_out/streams/bench_s$k.err || { tail -30 gpurun_out/streams/bench_s$k.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/streams/bench_s$k.json')); print($k, d['value'], d['hw_busy_pct'], d['pods_per_gpu'])"
done
for e in 1 2; do
  timeout -k 10 300 python tools/kbench.py --only modes --emulation spread --out gpurun_out/streams/modes.json > gpurun_out/streams/modes.log 2>&1 || { tail -30 gpurun_out/streams/modes.log; exit 1; }
  break
done
grep mode gpurun_out/streams/modes.log
