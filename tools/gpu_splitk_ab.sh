# same-box A/B: split-K + combine/LayerNorm allowed (default) vs fused-epilogue GEMM + LayerNorm only, whole bench
set -u
mkdir -p gpurun_out/sk
for rep in 1 2; do
  for sk in 1 0; do
    NOS_SPLITK=$sk timeout -k 10 300 python bench.py --no-density --out gpurun_out/sk/b_${sk}_$rep.json > /dev/null 2> gpurun_out/sk/b_${sk}_$rep.err || { tail -20 gpurun_out/sk/b_${sk}_$rep.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/sk/b_${sk}_$rep.json')); print('splitk $sk rep $rep', d['value'])"
  done
  for sk in 1 0; do
    NOS_SPLITK=$sk timeout -k 10 300 python tools/kbench.py --only modes --emulation spread --slices cpx --out gpurun_out/sk/m_${sk}_$rep.json > gpurun_out/sk/m_${sk}_$rep.log 2>&1 || { tail -20 gpurun_out/sk/m_${sk}_$rep.log; exit 1; }
    grep mode gpurun_out/sk/m_${sk}_$rep.log | python -c "import sys,json; [print('splitk $sk rep $rep', json.loads(l)['mode'], json.loads(l)['inf_per_s_per_gpu']) for l in sys.stdin]"
  done
done
