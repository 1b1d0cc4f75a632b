#!/bin/bash
# Memory-only (MPS-analogue) fairness variants on one MI355X: each variant runs the shared_5 and
# shared_7 scenarios of tools/multiproc.py as separate processes; stop at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
OUT=gpurun_out/multiproc_fair.json
ONLY=${NOS_FAIR_ONLY:-shared_5,shared_7}
# "<tag>|<env json>|<stagger s>"
for v in ${NOS_FAIR_VARIANTS:-'_q1|{"GPU_MAX_HW_QUEUES":"1"}|0'}; do
  IFS='|' read -r tag env stagger <<< "$v"
  timeout -k 10 300 python -u tools/multiproc.py --seconds 8 --only "$ONLY" --env "$env" --tag "$tag" \
    --stagger "$stagger" --out $OUT >> gpurun_out/multiproc_fair.log 2>&1 || { echo "variant $tag failed"; tail -20 gpurun_out/multiproc_fair.log; exit 1; }
done
grep scenario gpurun_out/multiproc_fair.log
