# x3 GEMM operand-load ablation at SPX (results invalid by design; timing only)
set -u
mkdir -p gpurun_out/r2ad
for ab in 0 1 2 3; do
  for spec in "qkv 14" "proj 24" "fc1 107" "fc2 24"; do set -- $spec
    NOS_X3_ABLATE=$ab timeout -k 10 300 python tools/contention.py --mode spx --ops $1 --tiles $2 --out gpurun_out/r2ad/ab${ab}_$1.json > /dev/null 2>&1 || exit 1
  done
done
