#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/serve
timeout -k 10 300 python -m pytest tests/test_serving_gpu.py -x -q > gpurun_out/serve/pytest.log 2>&1
rc=$?; tail -15 gpurun_out/serve/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python tools/bench_serve.py > gpurun_out/serve/bench.log 2>&1
rc=$?; cat gpurun_out/serve/bench.log | grep -v amdgpu.ids; exit $rc
