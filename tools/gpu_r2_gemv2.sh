#!/bin/bash
# Decode GEMV K split with the refined policy (deep K, no norm prologue): serving tests + decode bench A/B
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r2gemv2
mkdir -p $O
timeout -k 5 120 tools/kbench/bin/gemv_bench > $O/gemv.txt 2>&1 || exit $?
grep -E "wd|wqkv|wo " $O/gemv.txt | sed 's/skinny.*| gemv/gemv/'
timeout -k 10 300 python -u -m pytest tests/test_serving_gpu.py -x -q --timeout 200 --timeout-method thread > $O/pytest_serving.log 2>&1
rc=$?; tail -2 $O/pytest_serving.log; [ $rc -eq 0 ] || exit $rc
for ks in 1 0 1 0; do
  KFAMD_GEMV_KSPLIT=$ks timeout -k 10 300 python tools/bench_serve.py --batches 1,2,4,8 > $O/serve_ks$ks.log 2>&1
  rc=$?; echo "ksplit=$ks"; grep '"decode"' $O/serve_ks$ks.log; [ $rc -eq 0 ] || exit $rc
done
# dK/dV: spill fix alone vs spill fix + per-iteration lane constants
for r in 1 2; do
  for b in fa_new fa_remat; do
    echo "=== $b round $r" >> $O/fa.txt
    timeout -k 5 120 tools/kbench/bin/$b >> $O/fa.txt 2>&1 || exit $?
  done
done
grep -E "===|dkdv|NUMERICS" $O/fa.txt
