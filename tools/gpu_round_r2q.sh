# contention-tuned x3 GEMM tiles for DPX/QPX/CPX-sized slices (all eligible tiles, all siblings busy)
set -u
mkdir -p gpurun_out/r2q
cp walkai_nos_amd/ops/x3_tuned.json gpurun_out/r2q/x3_tuned.json
for m in cpx qpx dpx; do
  timeout -k 10 500 python tools/contention.py --mode $m --ops qkv,proj,fc1,fc2 --tiles all --emit-table gpurun_out/r2q/x3_tuned.json --out gpurun_out/r2q/tiles_$m.json > gpurun_out/r2q/tiles_$m.log 2>&1 || exit 1
done
timeout -k 10 300 python tools/contention.py --mode cpx --ops attn --head-blocks 6 --attn-groups 8,4 --out gpurun_out/r2q/attn_cpx.json > gpurun_out/r2q/attn_cpx.log 2>&1
