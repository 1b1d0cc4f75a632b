# per-mode throughput as the bench serves it (partitions wider than 64 CUs as 64-CU request lanes), twice
set -u
mkdir -p gpurun_out/ml
for rep in 1 2; do
  timeout -k 10 400 python tools/kbench.py --only modes --emulation spread --lane-cus 64 --out gpurun_out/ml/modes_$rep.json > gpurun_out/ml/modes_$rep.log 2>&1 || { tail -20 gpurun_out/ml/modes_$rep.log; exit 1; }
  grep mode gpurun_out/ml/modes_$rep.log | python -c "import sys,json; [print($rep, json.loads(l)['mode'], json.loads(l)['lanes_per_partition'], json.loads(l)['inf_per_s_per_gpu']) for l in sys.stdin]"
done
