# KFD per-process sysfs of a running HIP process (what is visible without root), then the CU guard
# test on real amd-smi (gpurun_out/cu_guard_samples.json)
set -u
mkdir -p gpurun_out
timeout -k 10 120 python3 - > gpurun_out/kfd_proc.txt 2>&1 <<'PY'
import os, subprocess, sys, time
p = subprocess.Popen([sys.executable, "-c", "import torch; x=torch.ones(10,device='cuda'); s=torch.cuda.Stream(); "
                      "print('up', flush=True); import time; time.sleep(5)"], stdout=subprocess.PIPE, text=True)
p.stdout.readline()
for root, dirs, files in os.walk(f"/sys/class/kfd/kfd/proc/{p.pid}"):
    for f in files:
        fp = os.path.join(root, f)
        try:
            v = open(fp).read().strip()[:200]
        except Exception as e:
            v = f"<{type(e).__name__}>"
        print(fp, "=", v)
p.wait()
PY
timeout -k 10 300 python -u -m pytest tests/test_gpu_native.py -x -v -rs -s --timeout 240 --timeout-method thread -k cu_guard > gpurun_out/cu_guard.log 2>&1
