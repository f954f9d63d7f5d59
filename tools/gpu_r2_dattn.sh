#!/bin/bash
# Decode attention with batched K loads (phase 1) and unrolled V streams (phase 3): tests + kernel/step bench
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r2dattn
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_serving_gpu.py -x -q --timeout 200 --timeout-method thread > $O/pytest_serving.log 2>&1
rc=$?; tail -2 $O/pytest_serving.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python tools/bench_serve.py --batches 1,8,32,64,128 > $O/serve.log 2>&1
rc=$?; grep -E '"decode|prefill' $O/serve.log; exit $rc
