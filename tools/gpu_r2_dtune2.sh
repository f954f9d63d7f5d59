#!/bin/bash
# Serving decode with the tuned decode-GEMM file vs hipBLASLt heuristics (B = 64, 128, 256), two rounds
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r2dtune2
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_serving_gpu.py -x -q --timeout 200 --timeout-method thread > $O/pytest_serving.log 2>&1
rc=$?; tail -2 $O/pytest_serving.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for t in 0 default; do
    if [ $t = 0 ]; then export KFAMD_DECODE_TUNED=0; else unset KFAMD_DECODE_TUNED; fi
    timeout -k 10 300 python tools/bench_serve.py --batches 64,128,256 --max-len 1280 > $O/serve_$t.$r.log 2>&1
    rc=$?; echo "tuned=$t round $r"; grep '"decode"' $O/serve_$t.$r.log; [ $rc -eq 0 ] || exit $rc
  done
done
