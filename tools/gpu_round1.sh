#!/bin/bash
# GPU session script: tests, bench, profile. Each GPU step has its own time limit.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1
echo "pytest rc=$?" 
tail -5 gpurun_out/pytest_gpu.log
timeout -k 10 400 python bench.py --steps 5 --warmup 2 --attn sdpa > gpurun_out/bench_sdpa.log 2>&1 || { echo bench failed; tail -20 gpurun_out/bench_sdpa.log; exit 1; }
tail -3 gpurun_out/bench_sdpa.log
