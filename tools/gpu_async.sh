#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/async
timeout -k 10 400 python -m pytest tests -x -q -m gpu > gpurun_out/async/pytest.log 2>&1
rc=$?; tail -3 gpurun_out/async/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 420 python bench.py --steps 10 --warmup 3 > gpurun_out/async/bench.log 2>&1
rc=$?; tail -1 gpurun_out/async/bench.log | cut -c1-330; [ $rc -eq 0 ] || exit $rc
