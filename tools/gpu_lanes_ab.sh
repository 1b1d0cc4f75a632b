# same-box A/B of request-lane widths (128 vs 64 CUs), alternated
set -u
mkdir -p gpurun_out/lab
for rep in 1 2; do
  for lc in 128 64; do
    timeout -k 10 300 python bench.py --no-density --lane-cus $lc --out gpurun_out/lab/b_${lc}_$rep.json > /dev/null 2> gpurun_out/lab/b_${lc}_$rep.err || { tail -20 gpurun_out/lab/b_${lc}_$rep.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/lab/b_${lc}_$rep.json')); print('lane_cus $lc rep $rep', d['value'], d['inference_latency_ms'])"
  done
done
