#!/bin/bash
# Kernel traces of steady-state replays on a 1/2 and a 1/8 slice (where the bench serves most pods)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/rp_slices
for s in dpx cpx; do
  (cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/rp_slices" \
    -o $s -- python3 "$GRAFT_REPO_ROOT/tools/model_replay.py" --slice $s --replays 20 > /dev/null 2>&1) || exit $?
  f=$(find gpurun_out/rp_slices -name "${s}_kernel_trace.csv" | sort | tail -1)
  python tools/replay_stats.py "$f" --replays 20 > gpurun_out/rp_slices/${s}_stats.txt 2>&1 || exit $?
done
