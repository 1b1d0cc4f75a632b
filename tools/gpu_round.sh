#!/bin/bash
# One GPU measurement round on the gpurun box: GPU tests, bench (HIP kernels and the PyTorch
# baseline backend), then a rocprofv3 kernel-trace profile of a short bench run.
# Every GPU step has its own time limit; a crash/fault/timeout stops the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$PWD
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
export TMPDIR=/tmp

step() {  # step <name> <timeout> <cmd...>: run, log, stop the round on fault/timeout
  local name=$1 to=$2; shift 2
  echo "== $name" | tee -a "$OUT/round.log"
  timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "   rc=$rc" | tee -a "$OUT/round.log"
  tail -5 "$OUT/$name.log" | tee -a "$OUT/round.log"
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then
    echo "stopping: $name ended with rc=$rc" | tee -a "$OUT/round.log"
    exit $rc
  fi
  return 0
}

: > "$OUT/round.log"
MODE=${1:-all}
if [ "$MODE" = all ] || [ "$MODE" = tests ]; then
  step pytest_gpu 900 python -m pytest tests -m gpu -q -rf
fi
if [ "$MODE" = all ] || [ "$MODE" = bench ]; then
  step bench_hip 600 python bench.py --steps 10 --warmup 2 --out "$OUT/bench_hip.json"
  step bench_torch 600 python bench.py --steps 10 --warmup 2 --backend torch --out "$OUT/bench_torch.json"
fi
if [ "$MODE" = all ] || [ "$MODE" = curve ]; then
  step sharing_curve 500 python tools/sharing_curve.py --seconds 4 --out "$OUT/sharing_curve.json"
fi
if [ "$MODE" = all ] || [ "$MODE" = prof ]; then
  cd /tmp
  step rocprof_bench 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o bench --output-format csv -- \
    python3 "$ROOT/bench.py" --steps 4 --warmup 1
fi
echo "round done" | tee -a "$OUT/round.log"
