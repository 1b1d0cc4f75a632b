# x3 GEMM ablation at SPX: operand loads (1 = A, 2 = W) and epilogue stores (4); timing only
set -u
mkdir -p gpurun_out/r2ae
for ab in 0 4 3 7; do
  for spec in "qkv 14" "proj 24" "fc1 107" "fc2 24"; do set -- $spec
    NOS_X3_ABLATE=$ab timeout -k 10 300 python tools/contention.py --mode spx --ops $1 --tiles $2 --out gpurun_out/r2ae/ab${ab}_$1.json > /dev/null 2>&1 || exit 1
  done
done
