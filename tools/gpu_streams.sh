# whole-GPU pod with 1, 2, 3 concurrent request streams (depth = inferences in flight per stream), same seed / window
set -u
mkdir -p gpurun_out/streams
for spec in "1 2" "2 1" "3 1" "2 2"; do
  set -- $spec
  timeout -k 10 400 python bench.py --pod-streams $1 --depth $2 --no-density > gpurun_out/streams/bench_s$1_d$2.json 2> gpurun_out/streams/bench.err || { tail -30 gpurun_out/streams/bench.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/streams/bench_s$1_d$2.json')); print('streams', $1, 'depth', $2, d['value'], d['hw_busy_pct'])"
done
