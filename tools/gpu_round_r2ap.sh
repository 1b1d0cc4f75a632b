# LayerNorm v2 (16-B row chunks): numerics, then same-box A/B vs v1 (SPX / CPX concurrent) and whole inference
set -u
mkdir -p gpurun_out/r2ap
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_kernels.py -k "layernorm or yolos" > gpurun_out/r2ap/pytest.log 2>&1 || exit 1
for v in 0 1; do
  NOS_LN_V2=$v timeout -k 10 300 python tools/contention.py --mode spx --ops ln --ln-wg-per-cu 1000 --out gpurun_out/r2ap/spx_v$v.json > /dev/null 2>&1 || exit 1
  NOS_LN_V2=$v timeout -k 10 300 python tools/contention.py --mode cpx --ops ln --ln-wg-per-cu 1000,4 --out gpurun_out/r2ap/cpx_v$v.json > /dev/null 2>&1 || exit 1
  NOS_LN_V2=$v timeout -k 10 300 python tools/model_replay.py --slice spx --replays 40 >> gpurun_out/r2ap/replay_v$v.log 2>&1 || exit 1
done
