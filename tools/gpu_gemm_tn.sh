#!/bin/bash
# Weight-gradient GEMM: numerics tests, microbench vs hipBLASLt, kernel profile.
set -o pipefail
mkdir -p gpurun_out/gemm_tn
python -c "from service_account_auth_improvements_amd.ops import _build; _build.build()" &&
timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py -q -x -k gemm_tn > gpurun_out/gemm_tn/pytest.log 2>&1 &&
timeout -k 10 300 python tools/bench_gemm_tn.py > gpurun_out/gemm_tn/bench.jsonl 2> gpurun_out/gemm_tn/bench.err
rc=$?
tail -5 gpurun_out/gemm_tn/pytest.log
cat gpurun_out/gemm_tn/bench.jsonl
exit $rc
