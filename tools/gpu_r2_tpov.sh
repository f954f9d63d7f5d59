#!/bin/bash
# GPU numerics after the async TP reductions: TP / TP+SP / CP / PP / DDP on the GPU kernels and the
# model-level tests.
set -o pipefail
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r2tpov
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_parallel_gpu.py tests/test_model_gpu.py tests/test_rccl_gpu.py -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; exit $rc
