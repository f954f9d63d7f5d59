#!/bin/bash
# dQ: -lse through the exp FMA (fa_l1) vs the folded MFMA (fa_l0), B4 S8192 32/8.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r3c_fa6
mkdir -p $O
for b in fa_l0 fa_l1 fa_l0 fa_l1 fa_l0 fa_l1; do
  echo "=== $b B4" >> $O/fa.txt
  timeout -k 5 120 tools/kbench/bin/$b 4 8192 32 8 10 1 >> $O/fa.txt 2>&1 || { echo "rc=$? on $b"; cat $O/fa.txt; exit 1; }
done
grep "===\|dq \|NUMERICS\|err" $O/fa.txt
