#!/bin/bash
# Round-end confirmation: full GPU test tier, then the default 1-GPU bench (the driver's N=1 config).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/final
timeout -k 10 400 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/final/pytest_gpu.log 2>&1
rc=$?; tail -2 gpurun_out/final/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 420 python bench.py > gpurun_out/final/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/final/bench.log; exit $rc
