#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/skinny
timeout -k 10 300 python -m pytest tests/test_serving_gpu.py -x -q -k skinny > gpurun_out/skinny/pytest.log 2>&1
rc=$?; tail -3 gpurun_out/skinny/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/bench_skinny.py 2>&1 | grep -v amdgpu.ids | tee gpurun_out/skinny/bench.log
