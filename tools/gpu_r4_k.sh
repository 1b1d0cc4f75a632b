#!/bin/bash
# Round-4 GPU batch: two-workgroups-per-CU x3 tiles (configs 39-42) — numerics on every shape and
# split count, then SPX / DPX / CPX model replays with and without them (interleaved), with the
# tuner's timings.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/wg2
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_kernels.py -x -v -k "gemm_x3 or splitk or linear_residual" \
  --timeout 300 --timeout-method thread > gpurun_out/wg2/pytest.log 2>&1
rc=$?; echo "gemm tests rc=$rc"; tail -4 gpurun_out/wg2/pytest.log; [ $rc -eq 0 ] || exit $rc
for rep in a b; do
  for sl in spx dpx; do
    for v in off on; do
      if [ $v = off ]; then drop=39,40,41,42; else drop=; fi
      NOS_X3_DROP=$drop timeout -k 10 200 python -u tools/model_replay.py --slice $sl --replays 200 --tables \
        > gpurun_out/wg2/${sl}_${v}_${rep}.log 2>&1
      rc=$?; echo "$sl wg2=$v $rep rc=$rc: $(grep 'per inference' gpurun_out/wg2/${sl}_${v}_${rep}.log)"; [ $rc -eq 0 ] || exit $rc
    done
  done
done
rm -f gpurun_out/multiproc_fair.json gpurun_out/multiproc_fair.log
NOS_FAIR_ONLY=shared_5,shared_7 NOS_FAIR_VARIANTS='_q3a|{"GPU_MAX_HW_QUEUES":"3"}|0 _q3b|{"GPU_MAX_HW_QUEUES":"3"}|0' \
  bash tools/gpu_fair.sh
