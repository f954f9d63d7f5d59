#!/bin/bash
# TunableOp: tune the fwd/dX GEMMs, then A/B the training bench (heuristic vs tuned file).
set -o pipefail
mkdir -p gpurun_out/tune
timeout -k 10 900 python -u tools/tune_gemm.py gpurun_out/tune/tunableop_gfx950.csv > gpurun_out/tune/tune.log 2>&1
rc=$?; cat gpurun_out/tune/tune.log | grep -v amdgpu; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 6 --warmup 2 > gpurun_out/tune/bench_default.log 2>&1 || exit 1
tail -1 gpurun_out/tune/bench_default.log | cut -c1-200
PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=0 PYTORCH_TUNABLEOP_FILENAME=gpurun_out/tune/tunableop_gfx950.csv \
  timeout -k 10 300 python bench.py --steps 6 --warmup 2 > gpurun_out/tune/bench_tuned.log 2>&1 || exit 1
tail -1 gpurun_out/tune/bench_tuned.log | cut -c1-200
