#!/bin/bash
# Round-4 GPU batch: the projection/fc2 tuner's timings of every pipeline (SPX, DPX), memory-only
# fairness (Allocate's one queue vs HIP's four), the ERQ bench and the default bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for sl in spx dpx; do
  timeout -k 10 200 python -u tools/model_replay.py --slice $sl --replays 100 --tables > gpurun_out/tables_$sl.log 2>&1
  rc=$?; echo "replay $sl rc=$rc"; grep "per inference" gpurun_out/tables_$sl.log; [ $rc -eq 0 ] || exit $rc
done
rm -f gpurun_out/multiproc_fair.json gpurun_out/multiproc_fair.log
NOS_FAIR_ONLY=shared_3,shared_5,shared_7,cumask_5,cumask_7 NOS_FAIR_VARIANTS='_alloc|{}|0 _q4|{"GPU_MAX_HW_QUEUES":"4"}|0' \
  bash tools/gpu_fair.sh || exit 1
timeout -k 10 300 python -u bench.py --erq --out gpurun_out/bench_erq_slices.json > gpurun_out/bench_erq_slices.log 2>&1
rc=$?; echo "erq rc=$rc"; tail -c 1200 gpurun_out/bench_erq_slices.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --out gpurun_out/bench_default.json > gpurun_out/bench_default.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -c 600 gpurun_out/bench_default.log; exit $rc
