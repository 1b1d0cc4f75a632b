#!/bin/bash
# The default bench over longer windows (100 and 200 quanta = 25 and 50 mean pod lifetimes)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u bench.py --steps 100 --warmup 5 --out gpurun_out/bench_r4_100q.json > gpurun_out/bench_r4_100q.log 2>&1 &&
timeout -k 10 500 python -u bench.py --steps 200 --warmup 5 --out gpurun_out/bench_r4_200q.json > gpurun_out/bench_r4_200q.log 2>&1
