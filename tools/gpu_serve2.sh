#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/serve2
timeout -k 10 300 python -m pytest tests/test_serving_gpu.py -x -q > gpurun_out/serve2/pytest.log 2>&1
rc=$?; tail -3 gpurun_out/serve2/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python tools/bench_serve.py --batches 1,4,8,16,32,64,128 2>&1 | grep -v amdgpu.ids | tee gpurun_out/serve2/bench.log
