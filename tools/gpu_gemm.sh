#!/bin/bash
# hipBLASLt heuristic vs TunableOp-tuned solutions for every Llama-3-8B training GEMM.
set -o pipefail
mkdir -p gpurun_out/gemm
timeout -k 10 200 python tools/bench_gemm.py > gpurun_out/gemm/default.log 2>&1 || exit 1
cat gpurun_out/gemm/default.log
PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_VERBOSE=0 \
PYTORCH_TUNABLEOP_FILENAME=gpurun_out/gemm/tunableop_results%d.csv \
PYTORCH_TUNABLEOP_MAX_TUNING_DURATION_MS=30 PYTORCH_TUNABLEOP_MAX_TUNING_ITERATIONS=10 \
  timeout -k 10 900 python tools/bench_gemm.py > gpurun_out/gemm/tuned.log 2>&1 || exit 1
cat gpurun_out/gemm/tuned.log
