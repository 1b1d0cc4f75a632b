#!/bin/bash
# Round-4 GPU batch: memory-only fairness, repeated (the per-pipe dispatch makes single runs noisy):
# Allocate's default (one hardware queue per pod) three times, two queues twice, at 3/5/7 pods.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -f gpurun_out/multiproc_fair.json gpurun_out/multiproc_fair.log
NOS_FAIR_ONLY=shared_3,shared_5,shared_7 \
NOS_FAIR_VARIANTS='_q1a|{}|0 _q2a|{"GPU_MAX_HW_QUEUES":"2"}|0 _q1b|{}|0 _q2b|{"GPU_MAX_HW_QUEUES":"2"}|0 _q1c|{}|0' \
  bash tools/gpu_fair.sh
