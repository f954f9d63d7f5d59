#!/bin/bash
# one-shot IPC all-reduce test (2 ranks sharing the GPU) under its own time limit
set -o pipefail
mkdir -p gpurun_out/car
timeout -k 10 300 python -u -m pytest tests/test_custom_ar_gpu.py tests/test_serving_tp_gpu.py -x -v --timeout 280 --timeout-method thread > gpurun_out/car/pytest.log 2>&1
rc=$?; tail -15 gpurun_out/car/pytest.log; exit $rc
