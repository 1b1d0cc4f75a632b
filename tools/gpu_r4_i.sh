#!/bin/bash
# Round-4 GPU batch: the staggered 8-wave GEMM tile (config 38, gemm_x3t) — numerics on every shape
# and split count, then SPX / DPX model replays with and without it (A/B, interleaved), with the
# tuner's timings.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/stagger
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -x -v -k "gemm_x3 or splitk or linear_residual" \
  --timeout 200 --timeout-method thread > gpurun_out/stagger/pytest.log 2>&1
rc=$?; echo "gemm tests rc=$rc"; tail -4 gpurun_out/stagger/pytest.log; [ $rc -eq 0 ] || exit $rc
for rep in a b; do
  for sl in spx dpx; do
    for v in off on; do
      if [ $v = off ]; then drop=38; else drop=; fi
      NOS_X3_DROP=$drop timeout -k 10 200 python -u tools/model_replay.py --slice $sl --replays 200 --tables \
        > gpurun_out/stagger/${sl}_${v}_${rep}.log 2>&1
      rc=$?; echo "$sl stagger=$v $rep rc=$rc: $(grep 'per inference' gpurun_out/stagger/${sl}_${v}_${rep}.log)"; [ $rc -eq 0 ] || exit $rc
    done
  done
done
