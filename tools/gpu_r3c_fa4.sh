#!/bin/bash
# forward K-read pipelining depth A/B; then bench with and without the dQ || dK/dV fork.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r3c_fa4
mkdir -p $O
for b in fa_f0 fa_f2 fa_f3 fa_f4 fa_f0 fa_f2 fa_f3 fa_f4; do
  echo "=== $b B4" >> $O/fa.txt
  timeout -k 5 120 tools/kbench/bin/$b 4 8192 32 8 10 1 >> $O/fa.txt 2>&1 || { echo "rc=$? on $b"; cat $O/fa.txt; exit 1; }
done
grep "===\|fwd\|NUMERICS" $O/fa.txt
for f in 1 0 1 0; do
  KFAMD_FA_BWD_FORK=$f timeout -k 10 600 python -u bench.py --steps 12 --warmup 4 --crd-jobs 0 > $O/bench_fork$f.log 2>&1 || { echo "bench rc=$?"; tail -30 $O/bench_fork$f.log; exit 1; }
  echo "fork=$f $(tail -1 $O/bench_fork$f.log | cut -c1-200)"
done
