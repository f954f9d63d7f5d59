#!/bin/bash
# dK/dV split-chain variants (read-ahead PA, s_setprio) vs the unsplit body, B4 S8192 32/8.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r3c_fa3
mkdir -p $O
for b in fa_ns fa_s1 fa_s2 fa_s2p fa_s3 fa_ns fa_s1 fa_s2 fa_s2p fa_s3; do
  echo "=== $b B4" >> $O/fa.txt
  timeout -k 5 120 tools/kbench/bin/$b 4 8192 32 8 10 1 >> $O/fa.txt 2>&1 || { echo "rc=$? on $b"; cat $O/fa.txt; exit 1; }
done
grep "===\|dkdv\|NUMERICS" $O/fa.txt
