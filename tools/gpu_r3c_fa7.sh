#!/bin/bash
# dK/dV transposed-fragment read-ahead 3 vs 4, B4 S8192 32/8.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r3c_fa7
mkdir -p $O
for b in fa_pt3 fa_pt4 fa_pt3 fa_pt4 fa_pt3 fa_pt4; do
  echo "=== $b B4" >> $O/fa.txt
  timeout -k 5 120 tools/kbench/bin/$b 4 8192 32 8 10 1 >> $O/fa.txt 2>&1 || { echo "rc=$? on $b"; cat $O/fa.txt; exit 1; }
done
grep "===\|dkdv\|NUMERICS" $O/fa.txt
