# same-box A/B: inferences in flight per request lane (2 vs 3), alternated
set -u
mkdir -p gpurun_out/dep
for rep in 1 2; do
  for d in 2 3; do
    timeout -k 10 300 python bench.py --no-density --depth $d --out gpurun_out/dep/b_${d}_$rep.json > /dev/null 2> gpurun_out/dep/b_${d}_$rep.err || { tail -20 gpurun_out/dep/b_${d}_$rep.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/dep/b_${d}_$rep.json')); print('depth $d rep $rep', d['value'], d['inference_latency_ms'])"
  done
done
