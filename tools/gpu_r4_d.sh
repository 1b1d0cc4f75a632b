#!/bin/bash
# Round-4 GPU batch: stream-K GEMM numerics + SPX/DPX model replay with and without it (+ the
# tuner's choices) + a kernel trace, then the suite, fairness with one hardware queue per pod, the
# ERQ bench and the default bench (tools/gpu_r4_c.sh).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -v -k "streamk or splitk or linear_residual" \
  --timeout 120 --timeout-method thread > gpurun_out/pytest_streamk.log 2>&1
rc=$?; echo "streamk tests rc=$rc"; tail -5 gpurun_out/pytest_streamk.log; [ $rc -eq 0 ] || exit $rc
for sl in spx dpx; do
  for v in 0 1; do
    NOS_STREAMK=$v timeout -k 10 200 python -u tools/model_replay.py --slice $sl --replays 200 --tables \
      > gpurun_out/replay_${sl}_sk$v.log 2>&1
    rc=$?; echo "replay $sl sk=$v rc=$rc: $(head -1 gpurun_out/replay_${sl}_sk$v.log)"; [ $rc -eq 0 ] || exit $rc
  done
done
mkdir -p gpurun_out/rp_sk
(cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/rp_sk" \
  -o spx -- python3 "$GRAFT_REPO_ROOT/tools/model_replay.py" --slice spx --replays 40 > /dev/null 2>&1)
rc=$?; echo "rocprof rc=$rc"; [ $rc -eq 0 ] || exit $rc
f=$(find gpurun_out/rp_sk -name "*kernel_trace.csv" | sort | tail -1)
[ -n "$f" ] && python tools/replay_stats.py "$f" --replays 40 > gpurun_out/rp_sk/spx_stats.txt 2>&1
head -16 gpurun_out/rp_sk/spx_stats.txt 2>/dev/null
exec_rc=0
bash tools/gpu_r4_c.sh || exec_rc=$?
exit $exec_rc
