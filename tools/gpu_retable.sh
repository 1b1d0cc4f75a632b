# re-measure the contention tile table for the model's qkv (fp32 out) and fc1 (planes out) GEMMs on
# concurrent CPX / QPX / DPX slices over every eligible tile (incl. the 256-wide 8-wave tiles)
set -u
mkdir -p gpurun_out/retable
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 200 --timeout-method thread -k "splitk" \
  > gpurun_out/retable/pytest.log 2>&1 || { tail -30 gpurun_out/retable/pytest.log; exit 1; }
tail -1 gpurun_out/retable/pytest.log
cp walkai_nos_amd/ops/x3_tuned.json gpurun_out/retable/x3_tuned.json
for mode in dpx qpx cpx; do
  timeout -k 10 500 python tools/contention.py --mode $mode --ops qkv_f32,fc1 --tiles all --iters 6 \
    --emit-table gpurun_out/retable/x3_tuned.json --out gpurun_out/retable/$mode.json > gpurun_out/retable/$mode.log 2>&1 || { tail -20 gpurun_out/retable/$mode.log; exit 1; }
  echo "$mode done"
done
python -c "
import json; d=json.load(open('gpurun_out/retable/x3_tuned.json'))
[print(k, v) for k, v in d.items()]"
