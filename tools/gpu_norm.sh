#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/norm
timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py -x -q > gpurun_out/norm/pytest.log 2>&1
rc=$?; tail -3 gpurun_out/norm/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/bench_norm.py 2>&1 | grep -v amdgpu.ids | tee gpurun_out/norm/bench.log
timeout -k 10 420 python bench.py --steps 8 --warmup 3 > gpurun_out/norm/bench_full.log 2>&1
rc=$?; tail -1 gpurun_out/norm/bench_full.log; exit $rc
