#!/bin/bash
# Batched prefill: GPU serving tests + prefill / decode bench (per-prompt vs batched prefill)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r2prefill
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_serving_gpu.py tests/test_serving_tp_gpu.py -x -q --timeout 200 --timeout-method thread > $O/pytest_serving.log 2>&1
rc=$?; tail -2 $O/pytest_serving.log; [ $rc -eq 0 ] || exit $rc
for pb in 4 16; do
  timeout -k 10 400 python tools/bench_serve.py --batches 1,8,64 --prefill-batch $pb > $O/serve_pb$pb.log 2>&1
  rc=$?; grep -E '"prefill|"decode"' $O/serve_pb$pb.log; [ $rc -eq 0 ] || exit $rc
done
