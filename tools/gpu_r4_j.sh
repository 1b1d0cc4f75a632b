#!/bin/bash
# Round-4 GPU batch: the committed tree as the driver runs it — GPU suite, smoke(), default bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/final
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/final/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/final/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -3 gpurun_out/final/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --out gpurun_out/final/bench.json > gpurun_out/final/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; grep -o '"value": [0-9.]*' gpurun_out/final/bench.log | head -1; exit $rc
