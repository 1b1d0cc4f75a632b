# per-slice kernel breakdown of one YOLOS-small inference (SPX and CPX) + per-kernel microbench
set -u
mkdir -p gpurun_out/r2l
export TMPDIR=/tmp
for sl in spx cpx; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/r2l_$sl -o m -- python3 tools/kbench.py --only model --slices $sl --iters 8 --out gpurun_out/r2l/model_$sl.json > gpurun_out/r2l/model_$sl.log 2>&1 || exit 1
  find /tmp/r2l_$sl -name "*kernel_stats.csv" -exec cp {} gpurun_out/r2l/model_${sl}_kernel_stats.csv \;
done
timeout -k 10 400 python tools/kbench.py --only gemm --slices spx,cpx --iters 20 --out gpurun_out/r2l/gemm.json > gpurun_out/r2l/gemm.log 2>&1 || exit 1
timeout -k 10 300 python tools/kbench.py --only attn --slices spx,cpx --iters 20 --out gpurun_out/r2l/attn.json > gpurun_out/r2l/attn.log 2>&1
