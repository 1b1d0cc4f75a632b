#!/bin/bash
# Round-4 GPU batch: the bench window on sliced GPUs for churn seeds 1-5 (measured seed spread next
# to the default seed 1234), then a kernel trace of a short bench run (kernel-busy share of the window).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/seeds_r4 gpurun_out/prof_r4
export TMPDIR=/tmp
for seed in 1 2 3 4 5; do
  timeout -k 10 240 python -u bench.py --no-density --seed $seed --out gpurun_out/seeds_r4/b_$seed.json \
    > gpurun_out/seeds_r4/b_$seed.log 2>&1
  rc=$?; echo "seed $seed rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/seeds_r4/b_$seed.log | head -1)"; [ $rc -eq 0 ] || exit $rc
done
(cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof_r4" \
  -o bench -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 6 --warmup 1 --no-density > "$GRAFT_REPO_ROOT/gpurun_out/prof_r4/bench.log" 2>&1)
rc=$?; echo "rocprof bench rc=$rc"; exit $rc
