#!/bin/bash
# Round-4 GPU batch: suite, fairness with one hardware queue per pod, ERQ bench, default bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
rm -f gpurun_out/multiproc_fair.json
NOS_FAIR_ONLY=shared_3,shared_5,shared_7,cumask_5,cumask_7,cpx8 NOS_FAIR_VARIANTS='_q1|{"GPU_MAX_HW_QUEUES":"1"}|0 _q4|{"GPU_MAX_HW_QUEUES":"4"}|0' bash tools/gpu_fair.sh || exit 1
timeout -k 10 300 python -u bench.py --erq --out gpurun_out/bench_erq_slices.json > gpurun_out/bench_erq_slices.log 2>&1
rc=$?; echo "erq rc=$rc"; tail -c 1500 gpurun_out/bench_erq_slices.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --out gpurun_out/bench_default.json > gpurun_out/bench_default.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -c 400 gpurun_out/bench_default.log; exit $rc
