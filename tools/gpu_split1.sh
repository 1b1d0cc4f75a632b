set -u
mkdir -p gpurun_out/split1
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q -k "gemm_x3" --timeout 240 --timeout-method thread > gpurun_out/split1/pytest.log 2>&1 || { tail -40 gpurun_out/split1/pytest.log; exit 1; }
tail -3 gpurun_out/split1/pytest.log
timeout -k 10 300 python tools/x3_shapes.py --out gpurun_out/split1/x3_shapes_spx.json > gpurun_out/split1/shapes.log 2>&1 || { tail -30 gpurun_out/split1/shapes.log; exit 1; }
cat gpurun_out/split1/shapes.log
