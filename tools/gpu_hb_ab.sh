# same-box A/B: attention heads per launch on 64-CU slices (rule: 3) vs all 6, through the whole bench
set -u
mkdir -p gpurun_out/hb
for rep in 1 2; do
  for hb in rule 6; do
    if [ $hb = rule ]; then unset NOS_ATTN_HEAD_BLOCK; else export NOS_ATTN_HEAD_BLOCK=$hb; fi
    timeout -k 10 300 python bench.py --no-density --out gpurun_out/hb/b_${hb}_$rep.json > /dev/null 2> gpurun_out/hb/b_${hb}_$rep.err || { tail -20 gpurun_out/hb/b_${hb}_$rep.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/hb/b_${hb}_$rep.json')); print('hb $hb rep $rep', d['value'], d['inference_latency_ms'])"
  done
done
unset NOS_ATTN_HEAD_BLOCK
timeout -k 10 300 python tools/kbench.py --only modes --emulation spread --slices qpx --out gpurun_out/hb/modes_rule.json > gpurun_out/hb/modes_rule.log 2>&1 || { tail -20 gpurun_out/hb/modes_rule.log; exit 1; }
NOS_ATTN_HEAD_BLOCK=6 timeout -k 10 300 python tools/kbench.py --only modes --emulation spread --slices qpx --out gpurun_out/hb/modes_6.json > gpurun_out/hb/modes_6.log 2>&1 || { tail -20 gpurun_out/hb/modes_6.log; exit 1; }
grep -h mode gpurun_out/hb/modes_rule.log gpurun_out/hb/modes_6.log
