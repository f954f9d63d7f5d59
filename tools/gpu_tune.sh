#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/tune
GEMM_SKIP=lm_head PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_FILENAME=gpurun_out/tune/tunableop_gfx950%d.csv \
PYTORCH_TUNABLEOP_MAX_TUNING_DURATION_MS=30 PYTORCH_TUNABLEOP_MAX_TUNING_ITERATIONS=30 \
  timeout -k 10 900 python tools/bench_gemm.py > gpurun_out/tune/tuned.log 2>&1 || exit 1
cat gpurun_out/tune/tuned.log
