#!/bin/bash
# A/B of the LayerNorm kernel's rows in flight per wave (NOS_LN_ROWS 1 vs 2): numerics, then
# whole-inference replays per slice, then kernel traces of a CPX replay for each. Ends at the first
# failing step (no retries).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$PWD
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q -k "layernorm" --timeout 120 \
  --timeout-method thread > "$OUT/ln_tests.log" 2>&1 || { tail -20 "$OUT/ln_tests.log"; exit 1; }
tail -2 "$OUT/ln_tests.log"
: > "$OUT/ln_ab.log"
for sl in spx dpx cpx; do
  for r in 1 2 1 2; do
    echo "slice=$sl rows=$r" >> "$OUT/ln_ab.log"
    NOS_LN_ROWS=$r timeout -k 10 200 python tools/model_replay.py --slice "$sl" --replays 200 >> "$OUT/ln_ab.log" 2>&1 \
      || { tail -20 "$OUT/ln_ab.log"; exit 1; }
  done
done
cat "$OUT/ln_ab.log"
for r in 1 2; do
  (cd /tmp && NOS_LN_ROWS=$r timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv \
     -d "$OUT/ln_prof_$r" -o cpx -- python3 "$ROOT/tools/model_replay.py" --slice cpx --replays 20) \
     > "$OUT/ln_prof_$r.log" 2>&1 || { tail -20 "$OUT/ln_prof_$r.log"; exit 1; }
done
echo done
