#!/bin/bash
# serving GPU tests + decode/prefill bench (Llama-3-8B, ctx 1024); first failure ends it.
set -o pipefail
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/serve}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_serving_gpu.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -5 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python tools/bench_serve.py --batches ${BATCHES:-1,4,8,16,32,64,128} > $OUT/bench.log 2>&1
rc=$?; grep -v amdgpu.ids $OUT/bench.log; exit $rc
