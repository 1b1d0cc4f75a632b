set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
echo "pytest rc=$?"; tail -3 gpurun_out/pytest_gpu.log
for v in '_s1|{}' '_s4|{"NOS_POD_STREAMS":"4"}' '_q2s4|{"NOS_POD_STREAMS":"4","GPU_MAX_HW_QUEUES":"2"}'; do
  tag=${v%%|*}; env=${v#*|}
  timeout -k 10 240 python -u tools/multiproc.py --seconds 8 --only shared_5,shared_7,cumask_5,cumask_7 --env "$env" --tag "$tag" --out gpurun_out/multiproc_fair.json >> gpurun_out/multiproc_fair.log 2>&1 || { echo "multiproc $tag failed rc=$?"; tail -20 gpurun_out/multiproc_fair.log; exit 1; }
done
grep scenario gpurun_out/multiproc_fair.log
