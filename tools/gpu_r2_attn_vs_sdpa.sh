#!/bin/bash
# HIP flash attention vs PyTorch-ROCm SDPA at the bench shape and at 32k tokens.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r2sdpa
timeout -k 10 300 python -u tools/bench_attn.py 2:8192 1:32768 4:8192 > gpurun_out/r2sdpa/attn.log 2>&1
rc=$?; cat gpurun_out/r2sdpa/attn.log | grep -v amdgpu.ids; exit $rc
