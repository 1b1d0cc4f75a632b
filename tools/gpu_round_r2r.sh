# new 96/192-wide x3 tiles: numerics, SPX timings, contention-tuned table, modes A/B
set -u
mkdir -p gpurun_out/r2r
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_kernels.py -k "gemm_x3" > gpurun_out/r2r/pytest.log 2>&1 || exit 1
timeout -k 10 400 python tools/kbench.py --only gemm --slices spx,dpx --iters 20 --out gpurun_out/r2r/gemm.json > gpurun_out/r2r/gemm.log 2>&1 || exit 1
echo '{}' > gpurun_out/r2r/x3_tuned.json
for m in cpx qpx dpx; do
  timeout -k 10 500 python tools/contention.py --mode $m --ops qkv,proj,fc1,fc2 --tiles all --emit-table gpurun_out/r2r/x3_tuned.json --out gpurun_out/r2r/tiles_$m.json > gpurun_out/r2r/tiles_$m.log 2>&1 || exit 1
done
cp gpurun_out/r2r/x3_tuned.json walkai_nos_amd/ops/x3_tuned.json
timeout -k 10 300 python tools/kbench.py --only modes --out gpurun_out/r2r/modes_tuned.json > gpurun_out/r2r/modes_tuned.log 2>&1 || exit 1
NOS_X3_TUNED=0 timeout -k 10 300 python tools/kbench.py --only modes --out gpurun_out/r2r/modes_untuned.json > gpurun_out/r2r/modes_untuned.log 2>&1
