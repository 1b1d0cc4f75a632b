#!/bin/bash
# HBM guard on real amd-smi accounting + the amd-smi tests, then a mode-rate refresh
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -s \
  tests/test_gpu_native.py -k "hbm_guard or amdsmi or hbm_limit" > gpurun_out/pytest_hbmguard_r4.log 2>&1 &&
timeout -k 10 400 python -u tools/kbench.py --only modes --free-s 5 --out gpurun_out/kbench_r4_modes.json > gpurun_out/kbench_r4_modes.log 2>&1
