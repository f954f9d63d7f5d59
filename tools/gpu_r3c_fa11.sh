#!/bin/bash
# dK/dV query rows per work item (QCH): 1024 (default) vs 1536 vs 2048, B4 and B2 S8192 32/8.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r3c_fa11
mkdir -p $O
for b in fa_q1024 fa_q1536 fa_q2048 fa_q1024 fa_q1536 fa_q2048; do
  echo "=== $b B4" >> $O/fa.txt
  timeout -k 5 120 tools/kbench/bin/$b 4 8192 32 8 10 1 >> $O/fa.txt 2>&1 || { echo "rc=$? on $b"; cat $O/fa.txt; exit 1; }
done
grep "===\|dkdv\|NUMERICS" $O/fa.txt
