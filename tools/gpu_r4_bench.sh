#!/bin/bash
# Round-4 bench comparison on one MI355X: the sliced layout (default) vs hardware partitions, a few
# churn seeds; each run under its own limit, stop at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {  # run <tag> <args...>
  local tag=$1; shift
  echo "== $tag $(date +%T)"
  timeout -k 10 300 python -u bench.py "$@" --out gpurun_out/bench_$tag.json > gpurun_out/bench_$tag.log 2>&1
  local rc=$?
  echo "   rc=$rc"; tail -c 600 gpurun_out/bench_$tag.log; echo
  [ $rc -eq 0 ] || exit $rc
}
# NOS_BENCH_RUNS: space-separated "<tag>:<arg>,<arg>..." entries
for spec in ${NOS_BENCH_RUNS:-slices_1234:--layout=slices partitions_1234:--layout=partitions}; do
  tag=${spec%%:*}; args=${spec#*:}
  run "$tag" ${args//,/ }
done
