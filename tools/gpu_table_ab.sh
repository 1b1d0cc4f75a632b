# same-box A/B of two x3 contention tables (a = current, b = candidate): per-mode throughput, alternated
set -u
mkdir -p gpurun_out/tab
for rep in 1 2 3 4; do
  for t in a b; do
    cp tools/x3_tuned_$t.json walkai_nos_amd/ops/x3_tuned.json
    timeout -k 10 400 python tools/kbench.py --only modes --emulation spread --slices cpx --out gpurun_out/tab/modes_${t}_$rep.json > gpurun_out/tab/modes_${t}_$rep.log 2>&1 || { tail -20 gpurun_out/tab/modes_${t}_$rep.log; exit 1; }
    grep mode gpurun_out/tab/modes_${t}_$rep.log | python -c "import sys,json; print('$t$rep', [(json.loads(l)['mode'][:3], json.loads(l)['inf_per_s_per_gpu']) for l in sys.stdin])"
  done
done
cp tools/x3_tuned_a.json walkai_nos_amd/ops/x3_tuned.json
