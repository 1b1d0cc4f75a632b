#!/bin/bash
# Round-4 GPU batch: memory-only fairness with Allocate's auto queue rule (2 queues up to 3
# memory-only slices, 1 beyond), twice at 3/4/5/7 pods, and the fairness GPU tests.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -f gpurun_out/multiproc_fair.json gpurun_out/multiproc_fair.log
NOS_FAIR_ONLY=shared_3,shared_4,shared_5,shared_7 NOS_FAIR_VARIANTS='_auto_a|{}|0 _auto_b|{}|0' \
  bash tools/gpu_fair.sh || exit 1
timeout -k 10 300 python -u -m pytest tests/test_gpu_native.py -x -v -k "share_compute_evenly" \
  --timeout 120 --timeout-method thread > gpurun_out/pytest_fair.log 2>&1
rc=$?; echo "fair tests rc=$rc"; tail -5 gpurun_out/pytest_fair.log; exit $rc
