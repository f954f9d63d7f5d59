#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/gemm
timeout -k 10 200 python tools/bench_gemm.py > gpurun_out/gemm/default.log 2>&1 || exit 1
cat gpurun_out/gemm/default.log
PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_FILENAME=gpurun_out/gemm/tunableop_results%d.csv \
PYTORCH_TUNABLEOP_MAX_TUNING_DURATION_MS=20 PYTORCH_TUNABLEOP_MAX_TUNING_ITERATIONS=20 \
  timeout -k 10 700 python tools/bench_gemm.py > gpurun_out/gemm/tuned.log 2>&1 || exit 1
cat gpurun_out/gemm/tuned.log
