#!/bin/bash
# GEMV K split also at 1-2 rows for K = 4096 (wo): serving GPU tests + decode bench B = 1, 2, 4
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r2gemv3
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_serving_gpu.py -x -q --timeout 200 --timeout-method thread > $O/pytest_serving.log 2>&1
rc=$?; tail -2 $O/pytest_serving.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  timeout -k 10 300 python tools/bench_serve.py --batches 1,2,4 --prefill-batch 1 > $O/serve.$r.log 2>&1
  rc=$?; grep '"decode"' $O/serve.$r.log; [ $rc -eq 0 ] || exit $rc
done
