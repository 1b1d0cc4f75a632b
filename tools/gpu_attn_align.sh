# A/B of the x3 attention grid rule (half-group alignment vs gcd alignment) on concurrent 64/32-CU slices and the bench
set -u
mkdir -p gpurun_out/al
for rep in 1 2; do
  for al in half gcd; do
    for mode in qpx cpx; do
      NOS_ATTN_ALIGN=$al timeout -k 10 300 python tools/contention.py --mode $mode --ops attn --head-blocks 6 --out gpurun_out/al/${mode}_${al}_$rep.json > gpurun_out/al/${mode}_${al}_$rep.log 2>&1 || { tail -20 gpurun_out/al/${mode}_${al}_$rep.log; exit 1; }
      grep -h op gpurun_out/al/${mode}_${al}_$rep.log | sed "s/^/$al $rep /"
    done
    NOS_ATTN_ALIGN=$al timeout -k 10 300 python bench.py --no-density --out gpurun_out/al/b_${al}_$rep.json > /dev/null 2> gpurun_out/al/b_${al}_$rep.err || { tail -20 gpurun_out/al/b_${al}_$rep.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/al/b_${al}_$rep.json')); print('bench $al $rep', d['value'])"
  done
done
