set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_native.py -m gpu -x -q --timeout 120 --timeout-method thread -k "probe" > gpurun_out/pytest_probe.log 2>&1
echo "pytest rc=$?"; tail -3 gpurun_out/pytest_probe.log
NOS_FAIR_VARIANTS='_s1|{}|0 _q1|{"GPU_MAX_HW_QUEUES":"1"}|0 _s4e|{"NOS_POD_STREAMS":"4","NOS_POD_EAGER_QUEUES":"1"}|0 _s4est|{"NOS_POD_STREAMS":"4","NOS_POD_EAGER_QUEUES":"1"}|2 _s1st|{}|2 _q2s2e|{"GPU_MAX_HW_QUEUES":"2","NOS_POD_STREAMS":"2","NOS_POD_EAGER_QUEUES":"1"}|0' bash tools/gpu_fair.sh
