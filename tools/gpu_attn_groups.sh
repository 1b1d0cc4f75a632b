# x3 attention query tiles per workgroup (4 vs 8) and heads per launch on concurrent CPX / QPX slices
set -u
mkdir -p gpurun_out/ag
for mode in cpx qpx; do
  timeout -k 10 300 python tools/contention.py --mode $mode --ops attn --attn-groups 4,8 --head-blocks 6,3 --out gpurun_out/ag/$mode.json > gpurun_out/ag/$mode.log 2>&1 || { tail -20 gpurun_out/ag/$mode.log; exit 1; }
  grep op gpurun_out/ag/$mode.log
done
