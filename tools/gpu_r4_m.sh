#!/bin/bash
# Density beyond 8 pods as processes: HIP's default queues for dedicated-CU slices vs one queue each
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u tools/multiproc.py --seconds 8 --only dense_14,shared_14 --out gpurun_out/dense_r4.json > gpurun_out/dense_r4.log 2>&1 &&
timeout -k 10 300 python -u tools/multiproc.py --seconds 8 --only dense_14 --env '{"GPU_MAX_HW_QUEUES": "1"}' --tag _q1 --out gpurun_out/dense_r4.json >> gpurun_out/dense_r4.log 2>&1 &&
timeout -k 10 300 python -u tools/multiproc.py --seconds 8 --only dense_14 --env '{"GPU_MAX_HW_QUEUES": "2"}' --tag _q2 --out gpurun_out/dense_r4.json >> gpurun_out/dense_r4.log 2>&1
