#!/bin/bash
# dK/dV spill fix A/B (standalone harness, alternating) + in-step bench with LM-head chunk 4096 / 8192
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r2s4ab
mkdir -p $O
for r in 1 2; do
  for b in fa_old fa_new; do
    echo "=== $b round $r" >> $O/fa.txt
    timeout -k 5 120 tools/kbench/bin/$b >> $O/fa.txt 2>&1
    rc=$?; if [ $rc -ne 0 ] && [ $rc -ne 3 ]; then echo "rc=$rc" >> $O/fa.txt; cat $O/fa.txt; exit $rc; fi
  done
done
cat $O/fa.txt
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > $O/bench_hc4096.log 2>&1
rc=$?; tail -1 $O/bench_hc4096.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --head-chunk 8192 > $O/bench_hc8192.log 2>&1
rc=$?; tail -1 $O/bench_hc8192.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -m pytest tests/test_attention_gpu.py -x -q --timeout 200 --timeout-method thread > $O/pytest_attn.log 2>&1
rc=$?; tail -2 $O/pytest_attn.log; exit $rc
