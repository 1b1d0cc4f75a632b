# persistent 256x128 tile: numerics, re-measured contention table (qkv fp32-out, fc1, proj, fc2), modes, bench
set -u
mkdir -p gpurun_out/rt2
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 300 --timeout-method thread -k "gemm_x3_every_tile" \
  > gpurun_out/rt2/pytest.log 2>&1 || { tail -30 gpurun_out/rt2/pytest.log; exit 1; }
tail -1 gpurun_out/rt2/pytest.log
cp walkai_nos_amd/ops/x3_tuned.json gpurun_out/rt2/x3_tuned.json
for mode in dpx qpx cpx; do
  timeout -k 10 500 python tools/contention.py --mode $mode --ops qkv_f32,fc1,proj,fc2 --tiles all --iters 6 \
    --emit-table gpurun_out/rt2/x3_tuned.json --out gpurun_out/rt2/$mode.json > gpurun_out/rt2/$mode.log 2>&1 || { tail -20 gpurun_out/rt2/$mode.log; exit 1; }
  echo "$mode done"
done
cp gpurun_out/rt2/x3_tuned.json walkai_nos_amd/ops/x3_tuned.json
timeout -k 10 400 python tools/kbench.py --only modes --emulation spread --out gpurun_out/rt2/modes.json > gpurun_out/rt2/modes.log 2>&1 || { tail -20 gpurun_out/rt2/modes.log; exit 1; }
grep mode gpurun_out/rt2/modes.log | python -c "import sys,json; [print(json.loads(l)['mode'], json.loads(l)['inf_per_s_per_gpu']) for l in sys.stdin]"
timeout -k 10 300 python bench.py --out gpurun_out/rt2/bench.json > /dev/null 2> gpurun_out/rt2/bench.err || { tail -20 gpurun_out/rt2/bench.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/rt2/bench.json')); print('bench', d['value'], d['inference_latency_ms'], d['density']['xcp'])"
