#!/bin/bash
# Per-slice GEMM timings the tuner measured (x3 tiles, fused linear+residual+LayerNorm pipelines)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for s in spx dpx cpx; do
  timeout -k 10 240 python -u tools/model_replay.py --slice $s --replays 20 --tables > gpurun_out/replay_tables_$s.log 2>&1 || exit $?
done
