#!/bin/bash
# Decode GEMV in-workgroup K split: harness A/B (KFAMD_GEMV_KSPLIT=1 = old grid) + serving tests + decode bench
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r2gemv
mkdir -p $O
for r in 1 2; do
  for ks in 1 0; do
    echo "=== KFAMD_GEMV_KSPLIT=$ks round $r" >> $O/gemv.txt
    KFAMD_GEMV_KSPLIT=$ks timeout -k 5 120 tools/kbench/bin/gemv_bench >> $O/gemv.txt 2>&1
    rc=$?; [ $rc -eq 0 ] || { echo "rc=$rc" >> $O/gemv.txt; cat $O/gemv.txt; exit $rc; }
  done
done
grep -E "===|gemv" $O/gemv.txt | grep -E "===|M=1|M=4" | head -60
timeout -k 10 300 python -u -m pytest tests/test_serving_gpu.py -x -q --timeout 200 --timeout-method thread > $O/pytest_serving.log 2>&1
rc=$?; tail -2 $O/pytest_serving.log; [ $rc -eq 0 ] || exit $rc
for ks in 1 0; do
  KFAMD_GEMV_KSPLIT=$ks timeout -k 10 300 python tools/bench_serve.py --batches 1,2,4,8 > $O/serve_ks$ks.log 2>&1
  rc=$?; echo "ksplit=$ks"; grep decode $O/serve_ks$ks.log; [ $rc -eq 0 ] || exit $rc
done
