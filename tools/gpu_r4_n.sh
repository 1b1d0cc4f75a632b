#!/bin/bash
# How many pod processes one GPU serves before the hardware scheduler time-slices processes
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u tools/multiproc.py --seconds 8 --only shared_8,shared_9,shared_10,shared_12 --out gpurun_out/procs_cap_r4.json > gpurun_out/procs_cap_r4.log 2>&1 &&
for f in /sys/class/kfd/kfd/topology/nodes/*/properties; do grep -H -E "simd_count|max_waves|num_cp_queues|num_xcc|cp_queue|vmid" $f || true; done > gpurun_out/kfd_props_r4.txt 2>&1
