#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/attn
timeout -k 10 300 python -m pytest tests/test_attention_gpu.py tests/test_kernels_gpu.py -x -q > gpurun_out/attn/pytest.log 2>&1
rc=$?; tail -3 gpurun_out/attn/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/bench_attn.py 4096 8192 2>&1 | grep -v amdgpu.ids | tee gpurun_out/attn/bench.log
