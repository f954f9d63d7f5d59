#!/bin/bash
# Round 3: GPU tests touched this round (dW GEMM ring, SwiGLU fallback, serving staging), then the bench.
set -o pipefail
O=gpurun_out/r3b2
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_kernels_gpu.py tests/test_serving_gpu.py tests/test_model_gpu.py > $O/pytest.log 2>&1 \
  || { echo "pytest rc=$?"; tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
timeout -k 10 600 python bench.py --steps 6 --warmup 2 --crd-jobs 0 > $O/bench.log 2>&1 || { echo "bench rc=$?"; tail -30 $O/bench.log; exit 1; }
tail -1 $O/bench.log
