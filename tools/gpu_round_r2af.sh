# packed x3-plane epilogue: numerics, run-to-run stress (incl. several workgroups per CU), timing
set -u
mkdir -p gpurun_out/r2af
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_kernels.py -k "gemm_x3 or yolos" > gpurun_out/r2af/pytest.log 2>&1 || exit 1
timeout -k 10 400 python tools/x3_gemm_stress.py --reps 10 > gpurun_out/r2af/stress.log 2>&1 || exit 1
for spec in "qkv 14" "qkv 7" "qkv 12" "fc1 14" "fc1 7" "fc1 107" "fc1 29"; do set -- $spec
  timeout -k 10 300 python tools/contention.py --mode spx --ops $1 --tiles $2 --out gpurun_out/r2af/$1_$2.json > /dev/null 2>&1 || exit 1
done
timeout -k 10 300 python tools/model_replay.py --slice spx --replays 40 > gpurun_out/r2af/replay.log 2>&1
