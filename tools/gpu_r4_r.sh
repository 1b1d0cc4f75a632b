#!/bin/bash
# Memory-only fairness at odd pod counts: mixed hardware-queue counts per pod (start order)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
O=gpurun_out/fair_mixq_r4.json
run() { timeout -k 10 200 python -u tools/multiproc.py --seconds 8 --only $1 --queues $2 --tag _q$(echo $2 | tr -d ,) --out $O >> gpurun_out/fair_mixq_r4.log 2>&1; }
run shared_5 1,2,1,2,1 && run shared_5 2,1,2,1,2 && run shared_5 2,2,2,2,1 && run shared_5 1,1,1,1,2 &&
run shared_7 1,2,1,2,1,2,1 && run shared_7 2,1,2,1,2,1,2
